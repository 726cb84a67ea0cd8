"""a13: NoisyLinear and the Rainbow dueling distributional head against
fixtures the reference's own code produced (tests/golden/gen_golden.py
gen_dueling: agilerl/modules/custom_components.py:38-131,
agilerl/networks/custom_modules.py:127-162 on create_mlp streams).  CPU, the
same torch ops: bit-exact."""

import numpy as np
import pytest
import torch


def test_noisy_linear_matches_reference(golden):
    from agilerl_amd.modules.custom_components import NoisyLinear

    g = golden("noisy0")
    torch.manual_seed(5)  # the reference's draw order: weight_mu, bias_mu uniforms, then eps_in, eps_out normals
    nl = NoisyLinear(12, 7, std_init=0.4)
    for k, v in nl.state_dict().items():
        assert np.array_equal(v.numpy(), g[f"init.{k}"]), k
    x = torch.from_numpy(g["x"])
    assert np.array_equal(nl(x).detach().numpy(), g["y_train"])
    nl.eval()
    assert np.array_equal(nl(x).detach().numpy(), g["y_eval"])
    nl.train()
    torch.manual_seed(9)
    nl.reset_noise()
    assert np.array_equal(nl.weight_epsilon.numpy(), g["w_eps2"])
    assert np.array_equal(nl.bias_epsilon.numpy(), g["b_eps2"])


@pytest.mark.parametrize("case", ["dueling0", "dueling1"])
def test_dueling_distributional_head_matches_reference(golden, case):
    from agilerl_amd.networks.q_networks import DuelingDistributionalMLP

    g = golden(case)
    L, A, Z = (int(v) for v in g["dims"])
    support = torch.from_numpy(g["support"])
    head = DuelingDistributionalMLP(num_inputs=L, num_outputs=A, hidden_size=[int(h) for h in g["hidden"]],
                                    num_atoms=Z, support=support, noisy=True, layer_norm=True, output_vanish=True,
                                    init_layers=False, noise_std=0.5)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    assert set(sd) == set(head.state_dict()), set(sd) ^ set(head.state_dict())
    head.load_state_dict(sd)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        assert np.array_equal(head(x).numpy(), g["q"])
        assert np.array_equal(head(x, q=False).numpy(), g["probs"])
        assert np.array_equal(head(x, log=True).numpy(), g["logp"])
    # the clamp(min=1e-3) is applied after the softmax and not renormalised (custom_modules.py:158)
    assert g["probs"].min() >= 1e-3
