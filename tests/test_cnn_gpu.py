"""Image path on the GPU: the HIP implicit-GEMM convolutions (csrc/conv.hip)
against fp32/fp64 ``torch.nn.functional.conv2d`` — the reference's
EvolvableCNN layers are plain ``nn.Conv2d`` (agilerl/utils/evolvable_networks.py:
263-318) — at the Atari encoder shapes; uint8 frames normalised inside the
first convolution vs the reference's ``(x - low) / (high - low)`` on f32
frames (algo_utils.py:1134-1183); EvolvableCNN / RainbowDQN learn vs a
plain-PyTorch twin of the same network; and config 3 (Pong Rainbow, pop 8,
2^20-leaf PER over a 1M-transition uint8 frame replay) for one generation.

Tolerances: the kernel sums the K = C*kh*kw products of an output in fp32
in an order different from torch's, and dW / db sum B*OH*OW products, so
results are compared to an fp64 CPU convolution within 2e-5 of the output's
scale (forward, dgrad) and 1e-5 of the gradient's scale (wgrad, db).
"""

import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (batch, C, H, W, OC, k, stride): ppo_image.yaml's Atari encoder
# (32/64/128, 8/4/3, 4/2/1), the default image encoder (32/32, 3/3, 1/1,
# evolvable_networks.py:190-196) and ragged shapes (odd channels, k > stride
# with a remainder, batch 1)
SHAPES = [
    (8, 4, 84, 84, 32, 8, 4),
    (8, 32, 20, 20, 64, 4, 2),
    (8, 64, 9, 9, 128, 3, 1),
    (4, 4, 84, 84, 32, 3, 1),
    (4, 32, 82, 82, 32, 3, 1),
    (1, 3, 17, 13, 5, 5, 3),
    (3, 7, 11, 11, 9, 2, 2),
    (2, 72, 12, 12, 40, 5, 1),  # K = 1800: gather tables rebuilt per 1024-entry chunk
    (2, 3, 14, 14, 6, 2, 3),    # k < stride: input phases no tap reaches (zero data gradient)
    (128, 64, 9, 9, 128, 3, 1),  # config 5's third layer at its batch: the dgrad split-K plan of the bench
]


def _scale(t: torch.Tensor) -> float:
    return max(float(t.detach().abs().max()), 1e-30)


def _close(got: torch.Tensor, want: torch.Tensor, rel: float, what: str) -> None:
    err = float((got.detach().double().cpu() - want.detach().double().cpu()).abs().max())
    assert err <= rel * _scale(want), f"{what}: max err {err:.3e} vs scale {_scale(want):.3e}"


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("relu", [False, True])
def test_conv_forward_backward_vs_torch(shape, relu):
    from agilerl_amd.modules.cnn import Conv2dFn

    B, C, H, W, OC, k, s = shape
    g = torch.Generator().manual_seed(SHAPES.index(shape))
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(OC, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(OC, generator=g) * 0.1
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = Conv2dFn.apply(xd, wd, bd, s, relu, None)
    # fp64 reference on the host
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, stride=s)
    if relu:
        yr = yr.relu()
    _close(y, yr, 2e-5, "forward")
    dy = torch.randn(yr.shape, generator=g)
    y.backward(dy.to(DEV))
    yr.backward(dy.double())
    _close(xd.grad, xr.grad, 2e-5, "dgrad")
    _close(wd.grad, wr.grad, 1e-5, "wgrad")
    _close(bd.grad, br.grad, 1e-5, "bias grad")


@pytest.mark.parametrize("low,high", [(0.0, 255.0), (-1.0, 7.0)])
def test_conv_uint8_frames_match_reference_normalisation(low, high):
    """u8 frames + in-kernel (x - low) / (high - low) == the f32 frames the
    reference normalises first (bit-identical inputs to the first conv, so the
    outputs agree as closely as the f32 path); dW / db through the u8 path."""
    from agilerl_amd.modules.cnn import Conv2dFn

    g = torch.Generator().manual_seed(11)
    frames = torch.randint(0, 256, (6, 4, 84, 84), generator=g, dtype=torch.uint8)
    w = (torch.randn(32, 4, 8, 8, generator=g) / 16).to(DEV).requires_grad_(True)
    b = (torch.randn(32, generator=g) * 0.1).to(DEV).requires_grad_(True)
    ref_in = (frames.float() - torch.tensor(low)) / (torch.tensor(high) - torch.tensor(low))
    y8 = Conv2dFn.apply(frames.to(DEV), w, b, 4, True, (low, high))
    w2, b2 = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yf = Conv2dFn.apply(ref_in.to(DEV), w2, b2, 4, True, None)
    assert torch.equal(y8, yf)  # same normalised values, same kernel order
    dy = torch.randn(y8.shape, generator=g).to(DEV)
    y8.backward(dy)
    yf.backward(dy)
    assert torch.equal(w.grad, w2.grad) and torch.equal(b.grad, b2.grad)
    with pytest.raises(ValueError):
        Conv2dFn.apply(frames.to(DEV), w, b, 4, True, None)


class _Gate(torch.nn.Module):
    """nn.ReLU whose gate can be pinned: with ``mask`` set, a grad-enabled
    forward multiplies by it instead of testing x > 0 (the HIP path's own
    ReLU gates replayed in the twin, so that a pre-activation lying within
    fp32 rounding of zero cannot gate differently in the two paths)."""

    def __init__(self):
        super().__init__()
        self.mask = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.mask is None or not torch.is_grad_enabled():
            return torch.relu(x)
        return x * self.mask


def _torch_twin(net, gates: bool = False):
    """The same network with plain nn.Conv2d + nn.ReLU modules (the reference's
    layers), weights copied; ``gates`` makes the conv ReLUs pinnable _Gates."""
    from agilerl_amd.modules.cnn import AgxConv2d, _FusedIdentity

    twin = copy.deepcopy(net)
    for mod in list(twin.modules()):
        for name, child in list(mod.named_children()):
            if isinstance(child, AgxConv2d):
                conv = torch.nn.Conv2d(child.in_channels, child.out_channels, child.kernel_size, child.stride,
                                       device=child.weight.device)
                conv.load_state_dict(child.state_dict())
                setattr(mod, name, conv)
            elif isinstance(child, _FusedIdentity):
                setattr(mod, name, _Gate() if gates else torch.nn.ReLU())
    return twin


ATARI_ENCODER = {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]}


def test_evolvable_cnn_matches_torch_twin():
    from agilerl_amd.modules import EvolvableCNN

    torch.backends.cudnn.allow_tf32 = False
    torch.manual_seed(5)
    net = EvolvableCNN([4, 84, 84], 256, device=DEV, output_activation="ReLU", **ATARI_ENCODER)
    twin = _torch_twin(net).double()
    assert list(net.state_dict()) == list(twin.state_dict())
    assert list(net.state_dict())[:2] == ["model.cnn_conv_layer_1.weight", "model.cnn_conv_layer_1.bias"]
    assert tuple(net.cnn_output_size) == (1, 128, 7, 7)
    frames = torch.randint(0, 256, (16, 4, 84, 84), dtype=torch.uint8, device=DEV)
    net.set_image_norm(0.0, 255.0)
    out = net(frames)
    ref = twin(frames.double() / 255.0)
    _close(out, ref, 2e-5, "EvolvableCNN forward")
    out.square().sum().backward()
    ref.square().sum().backward()
    for (n, p), q in zip(net.named_parameters(), twin.parameters()):
        _close(p.grad, q.grad, 5e-5, n)


def _atari_spaces():
    from agilerl_amd.envs import Box, Discrete

    return Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6)


@pytest.mark.parametrize("per", [False, True])
def test_rainbow_cnn_learn_matches_torch_twin(per):
    """RainbowDQN.learn with the Atari CNN encoder on uint8 frames vs the
    reference's learn (dqn_rainbow.py:284-490) on a plain-PyTorch twin fed
    the reference's normalised f32 frames."""
    from agilerl_amd.algorithms import RainbowDQN
    from test_dropin_gpu import _rainbow_reference_loss

    torch.backends.cudnn.allow_tf32 = False
    obs_space, act_space = _atari_spaces()
    torch.manual_seed(7)
    agent = RainbowDQN(obs_space, act_space, batch_size=32, lr=1e-4, gamma=0.99, tau=1e-3, v_min=-10, v_max=10,
                       num_atoms=51, net_config={"latent_dim": 64, "encoder_config": dict(ATARI_ENCODER),
                                                 "head_config": {"hidden_size": [64]}})
    assert agent.actor.encoder.model.encoder_conv_layer_1.image_norm == (0.0, 255.0)
    ref_actor, ref_target = _torch_twin(agent.actor), _torch_twin(agent.actor_target)
    ref_opt = torch.optim.Adam(ref_actor.parameters(), lr=1e-4)
    rng = np.random.default_rng(21 + int(per))
    B = 32
    exp = {"obs": rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8), "action": rng.integers(0, 6, (B, 1)),
           "reward": rng.choice([-1.0, 0.0, 1.0], (B, 1)).astype(np.float32),
           "next_obs": rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8),
           "done": (rng.random((B, 1)) < 0.2).astype(np.float32)}
    if per:
        exp["weights"] = rng.random((B, 1)).astype(np.float32)
        exp["idxs"] = np.arange(B).reshape(B, 1)
    ref_exp = dict(exp, obs=exp["obs"].astype(np.float32) / np.float32(255.0),
                   next_obs=exp["next_obs"].astype(np.float32) / np.float32(255.0))
    el_ref, loss_ref = _rainbow_reference_loss(agent, ref_actor, ref_target, ref_exp, 0.99, per)
    ref_opt.zero_grad()
    loss_ref.backward()
    ref_grads = [p.grad.clone() for p in ref_actor.parameters()]
    torch.nn.utils.clip_grad_norm_(ref_actor.parameters(), 10.0)
    ref_opt.step()
    loss, idxs, new_pri = agent.learn(exp, per=per)
    assert abs(loss - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())
    for (n, p1), g2 in zip(agent.actor.named_parameters(), ref_grads):  # .grad: unclipped (flat_state.py)
        _close(p1.grad, g2, 1e-4, n)
    # Adam's first step is ~lr * sign(g): parameters agree within 5 % of lr
    # wherever the gradient is well above the fp32 summation noise
    for (n, p1), p2 in zip(agent.actor.named_parameters(), ref_actor.parameters()):
        ok = p2.grad.abs() > 1e-3 * _scale(p2.grad)
        d = (p1 - p2).detach().abs()
        assert (float(d[ok].max()) if ok.any() else 0.0) <= 5e-6, n
        assert float(d.max()) <= 2.1e-4, n
    if per:
        np.testing.assert_allclose(new_pri, el_ref.detach().cpu().numpy() + agent.prior_eps, rtol=1e-5)
    acts = agent.get_action(exp["obs"], training=False)
    assert acts.shape == (B,) and ((acts >= 0) & (acts < 6)).all()


def test_config3_pong_rainbow_generation():
    """Config 3: pop 8 Rainbow DQN on 84x84x4 uint8 frames, a shared
    PrioritizedReplayBuffer of 1M transitions (2^20-leaf trees) + 3-step
    memory, frames stored as uint8 in HBM, 16 envs with N // learn_step = 16
    learns per vector step (train_off_policy.py:355-429), then evaluation and
    tournament selection — one generation."""
    from agilerl_amd.components import MultiStepReplayBuffer, PrioritizedReplayBuffer
    from agilerl_amd.envs import SyntheticAtariVecEnv
    from agilerl_amd.hpo.tournament import TournamentSelection
    from agilerl_amd.training import train_off_policy
    from agilerl_amd.utils import create_population

    obs_space, act_space = _atari_spaces()
    INIT_HP = {"BATCH_SIZE": 64, "LR": 1e-4, "LEARN_STEP": 1, "GAMMA": 0.99, "TAU": 1e-3, "N_STEP": 3,
               "BETA": 0.4, "PRIOR_EPS": 1e-6, "NUM_ATOMS": 51, "V_MIN": -200.0, "V_MAX": 200.0}
    net_config = {"latent_dim": 256, "min_latent_dim": 128, "max_latent_dim": 512,  # ppo_image.yaml:54-86
                  "encoder_config": dict(ATARI_ENCODER), "head_config": {"hidden_size": [256]}}
    torch.manual_seed(0)
    np.random.seed(0)
    from agilerl_amd.hpo.mutation import Mutations

    pop = create_population("Rainbow DQN", net_config, INIT_HP, obs_space, act_space, population_size=8)
    memory = PrioritizedReplayBuffer(1_000_000, alpha=0.6)
    n_mem = MultiStepReplayBuffer(1_000_000, n_step=3, gamma=0.99)
    assert memory.tree_capacity == 2 ** 20
    env = SyntheticAtariVecEnv(16, seed=3, p_done=1 / 50)
    p0 = [p.detach().clone() for p in pop[0].actor.parameters()]
    pop, fits = train_off_policy(env, "PongSynthetic", "Rainbow DQN", pop, memory, INIT_HP=INIT_HP,
                                 max_steps=128, evo_steps=128, eval_steps=40, eval_loop=1, per=True, n_step=True,
                                 n_step_memory=n_mem, learning_delay=64,
                                 tournament=TournamentSelection(2, True, 8, 1),
                                 mutation=Mutations(0.4, 0, 0.2, 0.3, 0, 0.3, rand_seed=3), verbose=False)
    assert len(fits) == 1 and len(fits[0]) == 8 and all(np.isfinite(fits[0]))
    st = memory.storage
    assert st["obs"].dtype == torch.uint8 and st["obs"].shape == (1_000_000, 4, 84, 84)
    assert st["next_obs"].dtype == torch.uint8
    assert 0 < len(memory) <= 8 * 128
    leaves = memory.sum_tree.tree[memory.tree_capacity:memory.tree_capacity + len(memory)]
    assert not torch.all(leaves == leaves[0])  # priorities updated from the C51 losses
    assert all(a.steps[-1] == 128 for a in pop)
    assert any(not torch.equal(a, b) for a, b in zip(p0, pop[0].actor.parameters()))

    # one more learn of the trained agent 0 on a PER batch drawn from the 1M-transition
    # memory, against the reference's loss (dqn_rainbow.py:284-440) on a plain-PyTorch
    # twin at the config-3 network (84x84x4 frames, latent 256, head [256], +-200)
    from test_dropin_gpu import _rainbow_reference_loss

    from agilerl_amd.modules.cnn import AgxConv2d

    torch.backends.cudnn.allow_tf32 = False
    agent = pop[0]
    ref_actor, ref_target = _torch_twin(agent.actor, gates=True), _torch_twin(agent.actor_target)
    # deep copies: Optimizer.load_state_dict keeps the tensors it is given, so a plain
    # load would let ref_opt.step() advance the AGENT's Adam moments and step count
    # (its exp_avg / exp_avg_sq are views of the agent's flat state) before its own
    # learn, which then applied a second moment update on top (the round-5 failure)
    state0 = copy.deepcopy(agent.optimizer.state_dict())
    ref_opt = torch.optim.Adam(ref_actor.parameters(), lr=agent.lr)
    ref_opt.load_state_dict(copy.deepcopy(state0))
    # torch's Adam replayed on the HIP path's own gradient, from the same state
    own = [torch.nn.Parameter(p.detach().clone()) for p in agent.actor.parameters()]
    own_opt = torch.optim.Adam(own, lr=agent.lr)
    own_opt.load_state_dict(copy.deepcopy(state0))

    # the HIP path's ReLU gates of every conv in learn's grad-enabled forward,
    # replayed in the twin: a pre-activation within fp32 rounding of zero then
    # gates alike in both paths, and every element of every gradient is held to
    # its summation-order bound below (no outlier allowance)
    hip_convs = [m for m in agent.actor.modules() if isinstance(m, AgxConv2d)]
    gates = [m for m in ref_actor.modules() if isinstance(m, _Gate)]
    assert len(hip_convs) == len(gates) and all(m.fuse_relu for m in hip_convs)
    masks = {}

    def grab(mod, inp, out):
        if torch.is_grad_enabled():
            assert mod not in masks  # one grad-enabled forward per learn
            masks[mod] = (out.detach() > 0).float()

    ghooks = [m.register_forward_hook(grab) for m in hip_convs]
    torch.manual_seed(11)
    exp = memory.sample(64, beta=0.4)
    loss, _, new_pri = agent.learn(exp, per=True)
    for h in ghooks:
        h.remove()
    assert len(masks) == len(hip_convs)
    for gate, conv in zip(gates, hip_convs):
        gate.mask = masks[conv]

    # a conv weight gradient sums 64 x OH x OW products of both signs: its fp32
    # error is bounded elementwise by the same sum over |input| x |grad output|
    seen = {}

    def keep(mod, inp, out):
        if torch.is_grad_enabled():
            seen[mod] = [inp[0].detach(), None]
            out.register_hook(lambda g, m=mod: seen[m].__setitem__(1, g.detach()))

    convs = [m for m in ref_actor.modules() if isinstance(m, torch.nn.Conv2d)]
    hooks = [m.register_forward_hook(keep) for m in convs]
    ref_exp = {k: (v.float() / 255.0 if k in ("obs", "next_obs") else v) for k, v in exp.items()}
    el_ref, loss_ref = _rainbow_reference_loss(agent, ref_actor, ref_target, ref_exp, agent.gamma, True)
    ref_opt.zero_grad()
    loss_ref.backward()
    for h in hooks:
        h.remove()
    clip = min(1.0, 10.0 / (float(torch.nn.utils.clip_grad_norm_(ref_actor.parameters(), 10.0)) + 1e-6))
    # below the top conv, grad output itself carries the rounding of the data
    # gradients above it: its conditioning is |grad output| propagated down
    # through |W| and the (pinned) ReLU gates (a summation-order change in any
    # dgrad moves it by that much, not by |grad output|)
    gyc = [None] * len(convs)
    gyc[-1] = seen[convs[-1]][1].abs()
    for i in range(len(convs) - 2, -1, -1):
        up = convs[i + 1]
        x_up = seen[up][0]
        prop = torch.nn.grad.conv2d_input(x_up.shape, up.weight.detach().abs(), gyc[i + 1], stride=up.stride)
        gyc[i] = torch.maximum(seen[convs[i]][1].abs(), prop * gates[i].mask)
    cond = {}
    for m, gc in zip(convs, gyc):
        x = seen[m][0]
        cond[id(m.weight)] = clip * torch.nn.grad.conv2d_weight(x.abs(), m.weight.shape, gc, stride=m.stride)
        cond[id(m.bias)] = clip * gc.sum((0, 2, 3))
    ref_opt.step()
    assert abs(loss - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())

    # (1) gradients vs the reference, every element within its bound
    hip_grads = [p.grad.detach().clone() for p in agent.actor.parameters()]
    bounds = []
    for (n, p1), p2, g in zip(agent.actor.named_parameters(), ref_actor.parameters(), hip_grads):
        g1 = g * clip  # .grad keeps the unclipped gradient (the clip is fused into Adam, flat_state.py)
        err = (g1.double() - p2.grad.double()).abs()
        if id(p2) in cond:
            bound = 1e-4 * cond[id(p2)].double() + 1e-7 * _scale(p2.grad)
        else:
            bound = torch.full_like(err, 1e-4 * _scale(p2.grad))
        bad = err > bound
        assert not bool(bad.any()), (n, int(bad.sum()), bad.nonzero()[:4].tolist(), err[bad][:4].tolist(),
                                     bound[bad][:4].tolist(), p2.grad[bad][:4].tolist(), g1[bad][:4].tolist())
        bounds.append(bound)

    # (2) the fused clip + Adam: the agent's new parameters == torch's Adam applied
    # to the HIP gradient with the agent's own clip coefficient (norm 10)
    norm = float(torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g.double()) for g in hip_grads])))
    own_clip = min(1.0, 10.0 / (norm + 1e-6))
    for q, g in zip(own, hip_grads):
        q.grad = g * own_clip
    own_opt.step()
    for (n, p1), q in zip(agent.actor.named_parameters(), own):
        d = (p1 - q).detach().abs()
        tol = 1e-3 * agent.lr + 1e-6 * q.detach().abs()
        assert bool((d <= tol).all()), (n, float(d.max()))

    # (3) vs the reference's parameters wherever the gradient's sign and size are
    # pinned by (1): |g| above 20x its bound moves Adam's step by < 5 % of lr
    for (n, p1), p2, bound in zip(agent.actor.named_parameters(), ref_actor.parameters(), bounds):
        det = p2.grad.double().abs() > 20 * bound
        d = (p1 - p2).detach().abs()
        assert (float(d[det].max()) if det.any() else 0.0) <= 0.05 * agent.lr, n
        assert float(d.max()) <= 2.1 * agent.lr, n
    np.testing.assert_allclose(new_pri, el_ref.detach().cpu().numpy() + agent.prior_eps, rtol=1e-5)


@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[1], SHAPES[2], SHAPES[5], SHAPES[8]])
def test_grouped_conv_matches_per_group_torch(shape):
    """agx_conv2d_*_grouped: G agents' convolutions in one launch, each agent's
    filters read in place from its row of a flat [G, n] buffer (row stride
    n > the filter size) == G separate fp64 convolutions."""
    from agilerl_amd.modules.cnn import Conv2dGroupedFn

    B, C, H, W, OC, k, s = shape
    G = 3
    g = torch.Generator().manual_seed(40 + SHAPES.index(shape))
    nw = OC * C * k * k
    flat = torch.randn(G, nw + OC + 7, generator=g) / (C * k * k) ** 0.5
    x = torch.randn(G, B, C, H, W, generator=g)
    flat_d = flat.to(DEV).requires_grad_(True)
    w = flat_d[:, :nw].view(G, OC, C, k, k)
    b = flat_d[:, nw:nw + OC]
    xd = x.to(DEV).requires_grad_(True)
    y = Conv2dGroupedFn.apply(xd, w, b, s, True, None)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(DEV))
    for p in range(G):
        xr = x[p].double().requires_grad_(True)
        wr = flat[p, :nw].view(OC, C, k, k).double().requires_grad_(True)
        br = flat[p, nw:nw + OC].double().requires_grad_(True)
        yr = torch.relu(F.conv2d(xr, wr, br, stride=s))
        yr.backward(gy[p].double())
        _close(y[p], yr, 2e-5, f"y[{p}]")
        _close(xd.grad[p], xr.grad, 2e-5, f"dx[{p}]")
        _close(flat_d.grad[p, :nw].view(OC, C, k, k), wr.grad, 1e-5, f"dw[{p}]")
        _close(flat_d.grad[p, nw:nw + OC], br.grad, 1e-5, f"db[{p}]")
    assert float(flat_d.grad[:, nw + OC:].abs().max()) == 0.0  # the rest of each row untouched
