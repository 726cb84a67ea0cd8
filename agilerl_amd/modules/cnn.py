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
        # dZ = dY * relu'(Y) once (one elementwise pass) instead of a second
        # (mask) load per gathered element in both the wgrad and the dgrad GEMM
        dy = (dy * (y > 0)).contiguous() if y is not None else dy.contiguous()
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


class EvolvableCNN(nn.Module):
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
        net = create_cnn(input_shape[0], channel_size, kernel_size, stride_size, name, init_layers, layer_norm,
                         activation, device)
        # flattened size (cnn.py:527-544), from the shapes
        c, h, w = input_shape
        for ch, k, s in zip(channel_size, kernel_size, stride_size):
            k = k[0] if isinstance(k, (tuple, list)) else k
            h, w, c = (h - k) // s + 1, (w - k) // s + 1, ch
        self.cnn_output_size = torch.Size([1, c, h, w])
        net[f"{name}_flatten"] = nn.Flatten()
        net[f"{name}_linear_output"] = nn.Linear(c * h * w, self.num_outputs, device=device)
        net[f"{name}_output_activation"] = get_activation(output_activation)
        self.model = nn.Sequential(net)

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

    def recreate_network(self) -> None:
        """Rebuild ``model`` from the current hyperparameters; parameters of
        equal name and shape are kept (preserve_parameters), as is the uint8
        normalisation of the first convolution."""
        from .mlp import preserve_parameters

        first = getattr(self.model, f"{self.name}_conv_layer_1")
        norm = first.image_norm
        dev = first.weight.device
        net = create_cnn(self.input_shape[0], self.channel_size, self.kernel_size, self.stride_size, self.name,
                         self.init_layers, self.layer_norm, self.activation, dev)
        c, h, w = self.cnn_output_size[1:]
        net[f"{self.name}_flatten"] = nn.Flatten()
        net[f"{self.name}_linear_output"] = nn.Linear(c * h * w, self.num_outputs, device=dev)
        net[f"{self.name}_output_activation"] = get_activation(self.output_activation)
        self.model = preserve_parameters(self.model, nn.Sequential(net))
        getattr(self.model, f"{self.name}_conv_layer_1").image_norm = norm

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(x, dtype=torch.float32, device=self.model[0].weight.device)
        if x.dim() == 3:  # missing batch dimension (cnn.py:577-578)
            x = x.unsqueeze(0)
        return self.model(x)
