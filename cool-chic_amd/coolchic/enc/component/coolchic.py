"""CoolChicEncoder (reference: coolchic/enc/component/coolchic.py).

Same constructor parameters, sub-modules and state_dict layout as the reference.
``forward`` in eval mode is the hot path, run entirely by libccmi HIP kernels:
  quantise + ARM context + MLP + Laplace rate -> ccmi_arm_forward_f32 (one launch),
  upsampling pyramid                           -> ccmi_ups_forward_f32 (one launch / level),
  synthesis                                    -> ccmi_syn_forward_f32 (one fused launch).
``forward_batch`` decodes many independent encoders (each with its own weights) of the
same size and architecture in one launch sequence; ``decoded_batch`` is the eval
FrameEncoder.forward through the fused decode kernel (no dense stack, no raw output).
"""

import math
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, OrderedDict, Sequence, Tuple

import torch
from torch import Tensor, nn

from ccmi import forward as _F
from coolchic.enc.component.core.arm import Arm, _get_non_zero_pixel_ctx_index
from coolchic.enc.component.core.synthesis import Synthesis
from coolchic.enc.component.core.upsampling import Upsampling

MAX_ARM_MASK_SIZE = 9


@dataclass
class CoolChicEncoderParameter:
    """coolchic.py:55-124."""

    layers_synthesis: List[str]
    n_ft_per_res: List[int]
    dim_arm: int = 24
    n_hidden_layers_arm: int = 2
    encoder_gain: int = 16
    ups_k_size: int = 8
    ups_preconcat_k_size: int = 7
    latent_n_grids: int = field(init=False)
    img_size: Optional[Tuple[int, int]] = field(init=False, default=None)

    def __post_init__(self):
        self.latent_n_grids = len(self.n_ft_per_res)

    def set_image_size(self, img_size: Tuple[int, int]) -> None:
        self.img_size = img_size

    def pretty_string(self) -> str:
        s = "CoolChicEncoderParameter value:\n-------------------------------\n"
        for k in fields(self):
            s += f"{k.name:<25}: {str(getattr(self, k.name)):<80}\n"
        return s + "\n"


@dataclass
class CoolChicEncoderOutput:
    raw_out: Tensor
    rate: Tensor
    additional_data: Dict[str, Any]


class CoolChicLatentGrid(nn.Module):
    """One latent resolution (coolchic.py:144-151)."""

    def __init__(self, data: torch.Tensor):
        super().__init__()
        self.data = nn.Parameter(data, requires_grad=True)


class CoolChicEncoder(nn.Module):
    """coolchic.py:154-795 (decode-side forward)."""

    def __init__(self, param: CoolChicEncoderParameter):
        super().__init__()
        self.param = param
        assert param.img_size is not None, "call param.set_image_size((H, W)) first"
        if any(c != 1 for c in param.n_ft_per_res):
            raise NotImplementedError("n_ft_per_res must be all 1 (as the reference decoder requires)")
        self.encoder_gains = param.encoder_gain
        self.size_per_latent = []
        self.latent_grids = nn.ModuleList()
        for i in range(param.latent_n_grids):
            h, w = [int(math.ceil(x / (2 ** i))) for x in param.img_size]
            self.size_per_latent.append((1, param.n_ft_per_res[i], h, w))
            self.latent_grids.append(CoolChicLatentGrid(torch.zeros(1, param.n_ft_per_res[i], h, w)))
        self.synthesis = Synthesis(sum(s[1] for s in self.size_per_latent), param.layers_synthesis)
        self.upsampling = Upsampling(param.ups_k_size, param.ups_preconcat_k_size, param.latent_n_grids - 1,
                                     param.latent_n_grids - 1)
        self.mask_size = MAX_ARM_MASK_SIZE
        self.register_buffer("non_zero_pixel_ctx_index", _get_non_zero_pixel_ctx_index(param.dim_arm),
                             persistent=False)
        self.arm = Arm(param.dim_arm, param.n_hidden_layers_arm)
        self.modules_to_send = ["arm", "upsampling", "synthesis"]

    @property
    def grid_sizes(self) -> List[Tuple[int, int]]:
        return [(s[2], s[3]) for s in self.size_per_latent]

    def flat_latent(self) -> Tensor:
        B = self.latent_grids[0].data.shape[0]
        return torch.cat([g.data.reshape(B, -1) for g in self.latent_grids], dim=1)

    def forward(self, quantizer_noise_type: str = "kumaraswamy", quantizer_type: str = "softround",
                soft_round_temperature: Optional[Tensor] = torch.tensor(0.3),
                noise_parameter: Optional[Tensor] = torch.tensor(1.0), AC_MAX_VAL: int = -1,
                flag_additional_outputs: bool = False) -> Tuple[Tensor, Tensor, Dict[str, Any]]:
        """coolchic.py:291-479: returns raw synthesis output [B, C, H, W], rate [B, N] in bits
        and the optional per-grid detail dictionary.  Eval mode: hard-rounded latents, no
        autograd (forward_batch).  Train mode: the reference's quantizer and noise
        (quantizer_type / quantizer_noise_type / soft_round_temperature / noise_parameter),
        differentiable w.r.t. every parameter; forward and backward both run in libccmi
        (ccmi.autograd.TrainForward), the noise drawn with the reference's torch calls."""
        if not self.training:
            return forward_batch([self], AC_MAX_VAL=AC_MAX_VAL, flag_additional_outputs=flag_additional_outputs)
        if AC_MAX_VAL != -1 or flag_additional_outputs:
            raise NotImplementedError("AC_MAX_VAL / additional outputs are eval-mode (bitstream) features")
        from ccmi import train as _T
        from ccmi.autograd import TrainForward
        from coolchic.enc.component.core.quantizer import draw_noise
        flat = self.flat_latent()
        if flat.device.type != "cuda":
            raise ValueError("CoolChicEncoder.forward runs on the GPU: move the module with .to('cuda')")
        # drawn whenever the reference draws it (quantizer.py:188-197), so the torch RNG stream
        # advances as in the reference; only "none" / "softround" add it (:200-213)
        noise = draw_noise(flat.detach() * self.encoder_gains, quantizer_noise_type, noise_parameter)
        p = self.param
        layers = tuple(self.synthesis.layer_desc)
        arch = _T.Arch(p.img_size[0], p.img_size[1], dim_arm=p.dim_arm, n_hidden=p.n_hidden_layers_arm, layers=layers,
                       n_grids=p.latent_n_grids, ups_k=p.ups_k_size, pre_k=p.ups_preconcat_k_size,
                       gain=float(self.encoder_gains))
        lin = [m for m in self.arm.mlp if hasattr(m, "weight")]
        convs = [m for m in self.synthesis.layers if hasattr(m, "weight")]
        params = _T.pack_params([(m.weight, m.bias) for m in lin],
                                [m.parametrizations.weight.original for m in self.upsampling.conv_transpose2ds],
                                [m.parametrizations.weight.original for m in self.upsampling.conv2ds],
                                [(m.weight, m.bias) for m in convs])
        t = float(soft_round_temperature) if soft_round_temperature is not None else 0.3
        raw, rate = TrainForward.apply(flat, params[None].expand(flat.shape[0], -1),
                                       {"arch": arch, "quantizer": quantizer_type, "temperature": t, "noise": noise})
        return raw, rate, {}

    # ---------------------------------------------------------------- parameters
    def get_param(self) -> "OrderedDict[str, Tensor]":
        return OrderedDict({k: v.detach().clone() for k, v in self.named_parameters()})

    def set_param(self, param) -> None:
        self.load_state_dict(param)

    def initialize_latent_grids(self, zeros: bool = True, random_seed: Optional[int] = None) -> None:
        g = None if zeros else torch.Generator().manual_seed(random_seed)
        for i, lat in enumerate(self.latent_grids):
            d = lat.data
            self.latent_grids[i] = CoolChicLatentGrid(
                torch.zeros_like(d) if zeros else 1e-2 * torch.randn(d.shape, generator=g))

    def reinitialize_parameters(self) -> None:
        self.arm.reinitialize_parameters()
        self.upsampling.reinitialize_parameters()
        self.synthesis.reinitialize_parameters()
        self.initialize_latent_grids()


def _check_same_arch(encs: Sequence[CoolChicEncoder]) -> None:
    p0 = encs[0].param
    for e in encs[1:]:
        p = e.param
        if (p.img_size, p.layers_synthesis, p.n_ft_per_res, p.dim_arm, p.n_hidden_layers_arm, p.ups_k_size,
                p.ups_preconcat_k_size, p.encoder_gain) != (p0.img_size, p0.layers_synthesis, p0.n_ft_per_res,
                                                            p0.dim_arm, p0.n_hidden_layers_arm, p0.ups_k_size,
                                                            p0.ups_preconcat_k_size, p0.encoder_gain):
            raise ValueError("forward_batch: all encoders must share image size and architecture")


def _batch_inputs(encs: Sequence[CoolChicEncoder], AC_MAX_VAL: int):
    """Flat latents [B, N] (AC_MAX_VAL-clamped integers when given), the per-frame packed
    parameter blocks, and the ARM's outputs: the common front of both eval paths."""
    _check_same_arch(encs)
    e0 = encs[0]
    dev = e0.latent_grids[0].data.device
    if dev.type != "cuda":
        raise ValueError("CoolChicEncoder.forward runs on the GPU: move the module with .to('cuda')")
    gain = float(e0.encoder_gains)
    flat = torch.cat([e.flat_latent() for e in encs], dim=0).float().contiguous()
    quantize = True
    if AC_MAX_VAL != -1:  # bitstream-writing clamp (coolchic.py:374-377)
        flat = torch.clamp(torch.round(flat * gain), -AC_MAX_VAL, AC_MAX_VAL + 1)
        quantize = False
    arm_p = torch.stack([e.arm.packed_params() for e in encs]).to(dev)
    ups_p = torch.stack([e.upsampling.packed_params() for e in encs]).to(dev)
    syn_p = torch.stack([e.synthesis.packed_params() for e in encs]).to(dev)
    return flat, quantize, gain, arm_p, ups_p, syn_p


@torch.no_grad()
def forward_batch(encs: Sequence[CoolChicEncoder], AC_MAX_VAL: int = -1, flag_additional_outputs: bool = False):
    """Eval forward of several independent CoolChicEncoders (own weights each) in one HIP launch
    sequence.  Returns (raw_out [B, C, H, W], rate [B, N], additional_data)."""
    flat, quantize, gain, arm_p, ups_p, syn_p = _batch_inputs(encs, AC_MAX_VAL)
    e0 = encs[0]
    sizes = e0.grid_sizes
    want = ("mu", "scale", "log_scale", "rate") if flag_additional_outputs else ("rate",)
    a = _F.arm_forward(flat, sizes, arm_p, e0.param.dim_arm, e0.param.n_hidden_layers_arm, gain, quantize, want)
    dense = e0.upsampling.forward_flat(flat, sizes, gain, quantize, params=ups_p)
    raw = e0.synthesis.forward(dense, params=syn_p)
    return raw, a["rate"], _additional(encs, flat, quantize, gain, a, flag_additional_outputs)


@torch.no_grad()
def decoded_batch(encs: Sequence[CoolChicEncoder], bitdepth: int, yuv420: bool, AC_MAX_VAL: int = -1,
                  flag_additional_outputs: bool = False, head: int = 0):
    """FrameEncoder.forward in eval mode (frame.py:153-183) for encoders whose architecture has
    a fused decode kernel: the ARM + rate (ccmi_arm_forward_f32), then ccmi_decode_forward_f32
    -- upsampling pyramid down to level 1, then ONE kernel for the last upsampling step,
    the synthesis and the post-processing (round to the bitdepth grid, 420, clamp), so the
    dense [L, H, W] stack and the raw synthesis output never reach HBM.  Returns (decoded
    [B, 3, H, W] or the flat 420 planes [B, H W + 2 (H/2)(W/2)], rate [B, N], additional
    data).  Raises CcmiError(ERR_UNSUPPORTED) for other architectures (forward_batch +
    post-processing then)."""
    flat, quantize, gain, arm_p, ups_p, syn_p = _batch_inputs(encs, AC_MAX_VAL)
    e0 = encs[0]
    p = e0.param
    sizes = e0.grid_sizes
    want = ("mu", "scale", "log_scale", "rate") if flag_additional_outputs else ("rate",)
    a = _F.arm_forward(flat, sizes, arm_p, p.dim_arm, p.n_hidden_layers_arm, gain, quantize, want)
    ups = e0.upsampling
    out = _F.decode_forward(flat, sizes, ups_p, ups.ups_k_size, ups.n_ups_kernel, ups.ups_preconcat_k_size,
                            ups.n_ups_preconcat_kernel, e0.synthesis.layer_desc, syn_p, gain, quantize, bitdepth,
                            yuv420, head)
    return out, a["rate"], _additional(encs, flat, quantize, gain, a, flag_additional_outputs)


def _additional(encs, flat, quantize, gain, a, flag_additional_outputs) -> Dict[str, Any]:
    """The per-grid detail dictionary of coolchic.py:426-479."""
    sizes = encs[0].grid_sizes
    add: Dict[str, Any] = {}
    if flag_additional_outputs:
        if len(encs) > 1:
            raise NotImplementedError("Batching is not yet supported for additional outputs.")
        q = flat if not quantize else torch.round(flat * gain)
        keys = ["detailed_sent_latent", "detailed_mu", "detailed_scale", "detailed_log_scale",
                "detailed_rate_bit", "detailed_centered_latent"]
        add = {k: [] for k in keys}
        add["hpfilters"] = []
        cnt = 0
        for h, w in sizes:
            sl = slice(cnt, cnt + h * w)
            lat = q[:, sl].view(1, 1, h, w)
            mu = a["mu"][:, sl].view(1, 1, h, w)
            add["detailed_sent_latent"].append(lat)
            add["detailed_mu"].append(mu)
            add["detailed_scale"].append(a["scale"][:, sl].view(1, 1, h, w))
            add["detailed_log_scale"].append(a["log_scale"][:, sl].view(1, 1, h, w))
            add["detailed_rate_bit"].append(a["rate"][:, sl].view(1, 1, h, w))
            add["detailed_centered_latent"].append(lat - mu)
            cnt += h * w
    return add
