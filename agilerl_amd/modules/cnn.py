"""Drop-in ``EvolvableCNN`` (agilerl/modules/cnn.py:224-552) whose Conv2d
layers run on the HIP implicit-GEMM kernels (csrc/conv.hip).

Same constructor arguments, module tree and state-dict keys as the reference
(``model.{name}_conv_layer_{i}.weight`` / ``.bias``, ``{name}_activation_{i}``,
``{name}_flatten``, ``{name}_linear_output``, ``{name}_output_activation``),
the same initialisation (conv layers: orthogonal gain sqrt(2), bias 0 via
layer_init, evolvable_networks.py:410-441; the final Linear keeps torch's
default init, cnn.py:536-540).  The parameters are ordinary ``nn.Conv2d`` /
``nn.Linear`` tensors; only the convolutions' forward and backward are ours
(``Conv2dFn``), fused with the layer's ReLU.

Image frames: when ``image_norm = (low, high)`` is set (the network does it
for an image Box space with finite bounds and normalize_images, algo_utils.py:
1134-1183), a uint8 batch is fed to the first convolution as is and each pixel
is normalised to (x - low) / (high - low) inside the kernel's load — the
replay / rollout storage keeps frames as uint8 in HBM and no f32 copy of the
batch is ever written.
"""

from __future__ import annotations

import ctypes
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from .. import _lib
from .mlp import get_activation, layer_init


class AgxConvShape(ctypes.Structure):
    """Mirror of ``agx_conv2d_shape`` (include/agx.h)."""

    _fields_ = [("batch", ctypes.c_int64), ("in_channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("out_channels", ctypes.c_int32), ("kernel_h", ctypes.c_int32),
                ("kernel_w", ctypes.c_int32), ("stride", ctypes.c_int32)]


def _shape(x: torch.Tensor, w: torch.Tensor, stride: int) -> AgxConvShape:
    s = AgxConvShape()
    s.batch, s.in_channels, s.height, s.width = x.shape
    s.out_channels, _, s.kernel_h, s.kernel_w = w.shape
    s.stride = int(stride)
    return s


class Conv2dFn(torch.autograd.Function):
    """y = relu?(conv2d(x, w, b, stride)) with agx_conv2d_forward /
    agx_conv2d_backward; x f32, or uint8 with ``norm = (low, high)``."""

    @staticmethod
    def forward(ctx, x, w, b, stride: int, relu: bool, norm):
        if x.device.type != "cuda":
            raise _lib.AgxError("Conv2dFn runs on the GPU (agx_conv2d_forward); no CPU fallback")
        u8 = x.dtype == torch.uint8
        if u8 and norm is None:
            raise ValueError("uint8 input needs image_norm = (low, high)")
        if not u8 and x.dtype != torch.float32:
            raise TypeError(f"conv input must be float32 or uint8, got {x.dtype}")
        x = x.contiguous()
        w = w.contiguous()
        sh = _shape(x, w, stride)
        OH = (sh.height - sh.kernel_h) // stride + 1
        OW = (sh.width - sh.kernel_w) // stride + 1
        y = torch.empty(x.shape[0], w.shape[0], OH, OW, dtype=torch.float32, device=x.device)
        lo, hi = (float(norm[0]), float(norm[1])) if u8 else (0.0, 1.0)
        _lib.call("agx_conv2d_forward", ctypes.byref(sh), x.data_ptr(), int(u8), lo, hi, w.data_ptr(),
                  _lib.ptr(b), int(relu), y.data_ptr(), _lib.stream())
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.meta = (stride, relu, u8, lo, hi, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        stride, relu, u8, lo, hi, has_b = ctx.meta
        sh = _shape(x, w, stride)
        dy = dy.contiguous()
        dw = torch.empty_like(w)
        db = torch.empty(w.shape[0], dtype=torch.float32, device=w.device) if has_b else None
        need_dx = ctx.needs_input_grad[0] and not u8
        dx = torch.empty_like(x) if need_dx else None
        ws = torch.empty(max(16, _lib.load().agx_conv2d_wgrad_workspace_bytes(ctypes.byref(sh))), dtype=torch.uint8,
                         device=w.device)
        _lib.call("agx_conv2d_backward", ctypes.byref(sh), x.data_ptr(), int(u8), lo, hi, w.data_ptr(),
                  _lib.ptr(y), dy.data_ptr(), _lib.ptr(dx), dw.data_ptr(), _lib.ptr(db), 0, ws.data_ptr(),
                  _lib.stream())
        return dx, dw, db, None, None, None


class Conv2dGroupedFn(torch.autograd.Function):
    """G independent convolutions of one shape in one launch (the population's
    agents): x [G, B, C, H, W] (f32, or uint8 with ``norm``), w [G, Cout, C, k,
    k] and b [G, Cout] whose groups may sit at any stride (views of rows of a
    flat [P, n] parameter buffer); -> y [G, B, Cout, OH, OW], relu fused.
    agx_conv2d_forward_grouped / agx_conv2d_backward_grouped."""

    @staticmethod
    def forward(ctx, x, w, b, stride: int, relu: bool, norm):
        if x.device.type != "cuda":
            raise _lib.AgxError("Conv2dGroupedFn runs on the GPU (agx_conv2d_forward_grouped); no CPU fallback")
        u8 = x.dtype == torch.uint8
        if u8 and norm is None:
            raise ValueError("uint8 input needs image_norm = (low, high)")
        if not u8 and x.dtype != torch.float32:
            raise TypeError(f"conv input must be float32 or uint8, got {x.dtype}")
        G = x.shape[0]
        x = x.contiguous()
        if w.shape[0] != G or b.shape[0] != G or not w[0].is_contiguous() or b.stride(1) != 1:
            raise ValueError("grouped conv: w [G, Cout, C, k, k] / b [G, Cout] with contiguous groups")
        sh = _shape(x[0], w[0], stride)
        OH = (sh.height - sh.kernel_h) // stride + 1
        OW = (sh.width - sh.kernel_w) // stride + 1
        y = torch.empty(G, x.shape[1], w.shape[1], OH, OW, dtype=torch.float32, device=x.device)
        lo, hi = (float(norm[0]), float(norm[1])) if u8 else (0.0, 1.0)
        _lib.call("agx_conv2d_forward_grouped", ctypes.byref(sh), G, x.data_ptr(), x[0].numel(), int(u8), lo, hi,
                  w.data_ptr(), w.stride(0), b.data_ptr(), b.stride(0), int(relu), y.data_ptr(), y[0].numel(),
                  _lib.stream())
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.meta = (stride, relu, u8, lo, hi)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        stride, relu, u8, lo, hi = ctx.meta
        G = x.shape[0]
        sh = _shape(x[0], w[0], stride)
        # dZ = dY * relu'(Y) once (one elementwise pass: ReLU's own backward
        # kernel, not a compare + cast + product) instead of a second (mask)
        # load per gathered element in both the wgrad and the dgrad GEMM
        dy = dy.contiguous()
        if y is not None:
            dy = torch.ops.aten.threshold_backward(dy, y, 0.0)
        dw = torch.empty((G, *w.shape[1:]), dtype=torch.float32, device=w.device)
        db = torch.empty(G, w.shape[1], dtype=torch.float32, device=w.device)
        need_dx = ctx.needs_input_grad[0] and not u8
        dx = torch.empty_like(x) if need_dx else None
        nws = _lib.load().agx_conv2d_wgrad_workspace_bytes_grouped(ctypes.byref(sh), G)
        ws = torch.empty(max(16, nws), dtype=torch.uint8, device=w.device)
        _lib.call("agx_conv2d_backward_grouped", ctypes.byref(sh), G, x.data_ptr(), x[0].numel(), int(u8), lo, hi,
                  w.data_ptr(), w.stride(0), None, dy.data_ptr(), dy[0].numel(), _lib.ptr(dx),
                  dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), _lib.stream())
        return dx, dw, db, None, None, None


class AgxConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state dict) whose forward is Conv2dFn;
    ``fuse_relu`` folds the following ReLU into the kernel epilogue."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size, stride, device=None):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, device=device)
        if self.kernel_size[0] != self.kernel_size[1] or self.stride[0] != self.stride[1]:
            raise NotImplementedError("agx conv layers: square kernels and strides (the EvolvableCNN Conv2d case)")
        self.fuse_relu = False
        self.image_norm = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return Conv2dFn.apply(x, self.weight, self.bias, int(self.stride[0]), self.fuse_relu,
                              self.image_norm if x.dtype == torch.uint8 else None)


class _FusedIdentity(nn.ReLU):
    """The activation after a conv whose kernel already applied it (keeps the
    reference's module name and type in the tree)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x


def create_cnn(in_channels: int, channel_size: list[int], kernel_size: list, stride_size: list[int],
               name: str = "cnn", init_layers: bool = True, layer_norm: bool = False, activation_fn: str = "ReLU",
               device="cpu") -> "OrderedDict[str, nn.Module]":
    """evolvable_networks.py:460-525 for Conv2d: conv (+ layer_init) ->
    activation per layer."""
    if layer_norm:
        raise NotImplementedError("BatchNorm2d between conv layers is outside the agx CNN path (layer_norm=False)")
    d: "OrderedDict[str, nn.Module]" = OrderedDict()
    chans = [in_channels, *channel_size]
    for i in range(1, len(chans)):
        k = kernel_size[i - 1]
        k = k[0] if isinstance(k, (tuple, list)) else k
        conv = AgxConv2d(chans[i - 1], chans[i], int(k), int(stride_size[i - 1]), device=device)
        if init_layers:
            conv = layer_init(conv)
        d[f"{name}_conv_layer_{i}"] = conv
        act = get_activation(activation_fn)
        if isinstance(act, nn.ReLU):
            conv.fuse_relu = True
            act = _FusedIdentity()
        d[f"{name}_activation_{i}"] = act
    return d


def max_kernel_sizes(kernel_size: list[int], channel_size: list[int], stride_size: list[int],
                     input_shape: list[int]) -> list[int]:
    """MutableKernelSizes.calc_max_kernel_sizes (modules/cnn.py:110-148): per
    layer a quarter of its output's smaller side (float arithmetic as the
    reference: np.floor of a true division), clamped to [1, 9]."""
    out = []
    h_in, w_in = input_shape[-2:]
    for idx, _ in enumerate(channel_size):
        h_out = 1 + np.floor((h_in + 2 * 0 - kernel_size[idx]) / stride_size[idx])
        w_out = 1 + np.floor((w_in + 2 * 0 - kernel_size[idx]) / stride_size[idx])
        k = int(min(h_out, w_out) * 0.25)
        out.append(1 if k <= 0 else (9 if k > 9 else k))
        h_in, w_in = h_out, w_out
    return out


def shrink_preserve_parameters(old_net: nn.Module, new_net: nn.Module) -> nn.Module:
    """EvolvableCNN.shrink_preserve_parameters (modules/cnn.py:418-456): equal
    shapes shared, otherwise the leading [:min0] / [:min0, :min1] block copied
    (spatial kernel dimensions are never sliced); norms left fresh."""
    old = dict(old_net.named_parameters())
    for key, param in new_net.named_parameters():
        if key in old:
            o = old[key]
            if o.data.size() == param.data.size():
                param.data = o.data
            elif "norm" not in key:
                m0 = min(o.data.size(0), param.data.size(0))
                if param.data.dim() == 1:
                    param.data[:m0] = o.data[:m0]
                else:
                    m1 = min(o.data.size(1), param.data.size(1))
                    param.data[:m0, :m1] = o.data[:m0, :m1]
    return new_net


class EvolvableCNN(nn.Module):
    """Architecture mutations (modules/cnn.py:582-760): ``add_layer`` /
    ``remove_layer`` (LAYER), ``change_kernel`` / ``add_channel`` /
    ``remove_channel`` (NODE), drawing from the module's ``rng`` as the
    reference's methods do (the kernel-size helper shares it), with the
    reference's fallbacks (add_layer -> add_channel at a limit or when the
    last output is too small; remove_layer -> add_channel at the minimum;
    change_kernel -> add_layer on a one-layer network).  As under the
    reference's MutationContext (modules/base.py:57-160), the network is
    recreated once, after the outermost method, with the outermost method's
    parameter copy (shrink for remove_layer / remove_channel); a fallback to
    a method the owner disabled (``disabled``: an EvolvableNetwork disables
    its encoder's LAYER methods, networks/base.py:266-268) applies nothing.
    ``last_mutation_attr`` names the method that actually ran."""

    LAYER_METHODS = ("add_layer", "remove_layer")
    NODE_METHODS = ("change_kernel", "add_channel", "remove_channel")

    def __init__(self, input_shape: list[int], num_outputs: int, channel_size: list[int], kernel_size: list,
                 stride_size: list[int], sample_input: torch.Tensor | None = None, block_type: str = "Conv2d",
                 activation: str = "ReLU", output_activation: str | None = None, min_hidden_layers: int = 1,
                 max_hidden_layers: int = 6, min_channel_size: int = 16, max_channel_size: int = 256,
                 layer_norm: bool = False, init_layers: bool = True, device="cpu", name: str = "cnn",
                 random_seed: int | None = None) -> None:
        super().__init__()
        assert len(kernel_size) == len(channel_size), \
            "Length of kernel size list must be the same length as channel size list."
        assert len(stride_size) == len(channel_size), \
            "Length of stride size list must be the same length as channel size list."
        assert num_outputs > 0, "'num_outputs' cannot be less than or equal to zero, please enter a valid integer."
        assert min_hidden_layers < max_hidden_layers, "'min_hidden_layers' must be less than 'max_hidden_layers."
        assert min_channel_size < max_channel_size, "'min_channel_size' must be less than 'max_channel_size'."
        if block_type != "Conv2d":
            raise NotImplementedError("agx EvolvableCNN: Conv2d blocks (the Atari encoders)")
        assert len(input_shape) == 3, f"For Conv2d, input_shape should be (channels, height, width), got {input_shape}"
        self.input_shape, self.num_outputs = list(input_shape), int(num_outputs)
        self.channel_size, self.kernel_size, self.stride_size = list(channel_size), list(kernel_size), list(stride_size)
        self.block_type, self.activation, self.output_activation = block_type, activation, output_activation
        self.min_hidden_layers, self.max_hidden_layers = min_hidden_layers, max_hidden_layers
        self.min_channel_size, self.max_channel_size = min_channel_size, max_channel_size
        self.layer_norm, self.init_layers, self.name, self.device = layer_norm, init_layers, name, device
        self.kernel_size = [int(k[0] if isinstance(k, (tuple, list)) else k) for k in self.kernel_size]
        self.random_seed = random_seed
        self.rng = np.random.default_rng(seed=random_seed)  # EvolvableModule.rng (modules/base.py)
        # MutableKernelSizes keeps the generator the CNN was built with (cnn.py:367-372):
        # an owner that shares its own generator into this module leaves it in place
        self.kernel_rng = self.rng
        self.last_mutation_attr: str | None = None
        self.disabled: set[str] = set()
        self._depth = 0
        self.model = self._build(device)

    def _build(self, device) -> nn.Sequential:
        """EvolvableCNN.create_cnn (modules/cnn.py:487-544): conv blocks, then
        flatten -> Linear(flattened, num_outputs) -> output activation; the
        flattened size follows from the shapes (the reference runs a sample
        input through the block — no random draws either way)."""
        net = create_cnn(self.input_shape[0], self.channel_size, self.kernel_size, self.stride_size, self.name,
                         self.init_layers, self.layer_norm, self.activation, device)
        c, h, w = self.input_shape
        for ch, k, s in zip(self.channel_size, self.kernel_size, self.stride_size):
            h, w, c = (h - k) // s + 1, (w - k) // s + 1, ch
        if h < 1 or w < 1:
            raise ValueError(f"EvolvableCNN: kernels {self.kernel_size} / strides {self.stride_size} leave no "
                             f"output for input {self.input_shape}")
        self.cnn_output_size = torch.Size([1, c, h, w])
        net[f"{self.name}_flatten"] = nn.Flatten()
        net[f"{self.name}_linear_output"] = nn.Linear(c * h * w, self.num_outputs, device=device)
        net[f"{self.name}_output_activation"] = get_activation(self.output_activation)
        return nn.Sequential(net)

    @property
    def net_config(self) -> dict:
        return dict(channel_size=self.channel_size, kernel_size=self.kernel_size, stride_size=self.stride_size,
                    activation=self.activation, output_activation=self.output_activation,
                    min_hidden_layers=self.min_hidden_layers, max_hidden_layers=self.max_hidden_layers,
                    min_channel_size=self.min_channel_size, max_channel_size=self.max_channel_size,
                    layer_norm=self.layer_norm, init_layers=self.init_layers)

    def set_image_norm(self, low: float, high: float) -> None:
        """uint8 batches are normalised to (x - low) / (high - low) inside the
        first convolution (preprocess_observation, algo_utils.py:1134-1183)."""
        first = getattr(self.model, f"{self.name}_conv_layer_1")
        first.image_norm = (float(low), float(high))

    def clear_image_norm(self) -> None:
        getattr(self.model, f"{self.name}_conv_layer_1").image_norm = None

    def change_activation(self, activation: str, output: bool = False) -> None:
        """modules/cnn.py:473-485: a new activation (and output activation
        when ``output``), the network recreated with its parameters kept."""
        if output:
            self.output_activation = activation
        self.activation = activation
        self.recreate_network()

    def recreate_network(self, shrink_params: bool = False) -> None:
        """Rebuild ``model`` from the current hyperparameters (cnn.py:769-790):
        parameters of equal name are kept, overlapping slices copied
        (shrink_preserve_parameters for shrinking mutations), as is the uint8
        normalisation of the first convolution."""
        from .mlp import preserve_parameters

        first = getattr(self.model, f"{self.name}_conv_layer_1")
        norm = first.image_norm
        dev = first.weight.device
        new = self._build(dev)
        self.model = (shrink_preserve_parameters if shrink_params else preserve_parameters)(self.model, new)
        getattr(self.model, f"{self.name}_conv_layer_1").image_norm = norm

    # ---- architecture mutations (modules/cnn.py:582-760) --------------------
    @property
    def mutation_methods(self) -> list[str]:
        return [m for m in (*self.LAYER_METHODS, *self.NODE_METHODS) if m not in self.disabled]

    def disable_mutations(self, kind: str | None = None) -> None:
        """EvolvableModule.disable_mutations: "layer", "node" or both (None)."""
        if kind in (None, "layer"):
            self.disabled.update(self.LAYER_METHODS)
        if kind in (None, "node"):
            self.disabled.update(self.NODE_METHODS)

    def _mutate(self, name: str, body, shrink: bool = False):
        """One mutation method under the MutationContext rules."""
        self._depth += 1
        self.last_mutation_attr = name
        try:
            if name in self.disabled:
                self.last_mutation_attr = None
                return None
            return body()
        finally:
            self._depth -= 1
            if self._depth == 0 and self.last_mutation_attr is not None:
                self.recreate_network(shrink_params=shrink)

    def add_layer(self):
        return self._mutate("add_layer", self._add_layer)

    def remove_layer(self):
        return self._mutate("remove_layer", self._remove_layer, shrink=True)

    def change_kernel(self, kernel_size: int | None = None, hidden_layer: int | None = None):
        return self._mutate("change_kernel", lambda: self._change_kernel(kernel_size, hidden_layer))

    def add_channel(self, hidden_layer: int | None = None, numb_new_channels: int | None = None):
        return self._mutate("add_channel", lambda: self._add_channel(hidden_layer, numb_new_channels))

    def remove_channel(self, hidden_layer: int | None = None, numb_new_channels: int | None = None):
        return self._mutate("remove_channel", lambda: self._remove_channel(hidden_layer, numb_new_channels),
                            shrink=True)

    def _add_layer(self):
        dims = self.cnn_output_size[-2:]
        maxk = max_kernel_sizes(self.kernel_size, self.channel_size, self.stride_size, self.input_shape)
        if len(self.channel_size) < self.max_hidden_layers and not any(i <= 2 for i in dims) and maxk \
                and maxk[-1] > 2:
            l_in = int(self.cnn_output_size[-1])
            if l_in < 2:
                return self.add_channel()
            k_new = int(self.rng.integers(2, l_in + 1))
            max_s = l_in - k_new + 1
            if max_s < 1:
                return self.add_channel()
            s_new = int(self.rng.integers(1, max_s + 1))
            self.channel_size = [*self.channel_size, self.channel_size[-1]]
            self.kernel_size = [*self.kernel_size, k_new]
            self.stride_size = [*self.stride_size, s_new]
            return None
        return self.add_channel()

    def _remove_layer(self):
        if len(self.channel_size) > self.min_hidden_layers:
            self.channel_size = self.channel_size[:-1]
            self.kernel_size = self.kernel_size[:-1]
            self.stride_size = self.stride_size[:-1]
            return None
        return self.add_channel()

    def _change_kernel(self, kernel_size, hidden_layer):
        if len(self.channel_size) > 1:
            if hidden_layer is None:
                hidden_layer = int(self.rng.integers(1, min(4, len(self.channel_size))))
            if kernel_size is not None:
                new_k = int(kernel_size)
            else:  # MutableKernelSizes.change_kernel_size (cnn.py:150-221)
                maxk = max_kernel_sizes(self.kernel_size, self.channel_size, self.stride_size,
                                        self.input_shape)[hidden_layer]
                cur = self.kernel_size[hidden_layer]
                if maxk == 1:
                    new_k = 1
                else:
                    cand = [k for k in range(1, maxk + 1) if k != cur]
                    new_k = int(self.kernel_rng.choice(cand)) if cand else \
                        int(self.kernel_rng.integers(1, maxk + 1))
            ks = list(self.kernel_size)
            ks[hidden_layer] = new_k
            self.kernel_size = ks
            return {"hidden_layer": hidden_layer, "kernel_size": new_k}
        return self.add_layer()

    def _add_channel(self, hidden_layer, numb):
        hidden_layer = int(self.rng.integers(0, len(self.channel_size))) if hidden_layer is None else \
            min(hidden_layer, len(self.channel_size) - 1)
        if numb is None:
            numb = int(self.rng.choice([8, 16, 32]))
        if self.channel_size[hidden_layer] + numb <= self.max_channel_size:
            ch = list(self.channel_size)
            ch[hidden_layer] += numb
            self.channel_size = ch
        return {"hidden_layer": hidden_layer, "numb_new_channels": numb}

    def _remove_channel(self, hidden_layer, numb):
        hidden_layer = int(self.rng.integers(0, len(self.channel_size))) if hidden_layer is None else \
            min(hidden_layer, len(self.channel_size) - 1)
        if numb is None:
            numb = int(self.rng.choice([8, 16, 32]))
        if self.channel_size[hidden_layer] - numb >= self.min_channel_size:
            ch = list(self.channel_size)
            ch[hidden_layer] -= numb
            self.channel_size = ch
        else:
            numb = 0
        return {"hidden_layer": hidden_layer, "numb_new_channels": numb}

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(x, dtype=torch.float32, device=self.model[0].weight.device)
        if x.dim() == 3:  # missing batch dimension (cnn.py:577-578)
            x = x.unsqueeze(0)
        return self.model(x)
