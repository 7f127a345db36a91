"""quantize_model on the GPU: the post-training search of one (weight, bias)
quantisation-step pair per network (enc/training/quantizemodel.py:120-302), with every
candidate of a module evaluated in ONE batched eval forward instead of one forward per
candidate (491 sequential forwards per frame in the reference).

Greedy over the modules in the reference's order (sorted names: arm, synthesis,
upsampling).  A candidate's loss is MSE(decoded, target) + lmbda * (latent rate + network
rate) / (H W) (loss.py); the network rate is exp_golomb_nbins at the best count
(misc.py:248-268).  Terms that do not depend on the module under search (the distortion
for the ARM, the latent rate for the synthesis / upsampling, the rate of the other
networks) are the same for every candidate and drop out of the argmin.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import ArmArgs, MAX_GRIDS, MAX_SYN_LAYERS, PostArgs, SynArgs, SynLayer, UpsArgs, check, lib
from .train import Arch

MAX_AC_MAX_VAL = 65535
POSSIBLE_Q_STEP = {  # misc.py POSSIBLE_Q_STEP
    "arm": {"weight": 2.0 ** np.linspace(-8, 0, 9), "bias": 2.0 ** np.linspace(-16, 0, 17)},
    "upsampling": {"weight": 2.0 ** np.linspace(-12, 0, 13), "bias": np.array([1.0])},
    "synthesis": {"weight": 2.0 ** np.linspace(-12, 0, 13), "bias": 2.0 ** np.linspace(-24, 0, 25)},
}
EXPGOL_COUNTS = np.arange(13)


def exp_golomb_nbins(sym: np.ndarray, count: int) -> float:
    """misc.py:248-268 (float32 arithmetic as torch does it)."""
    s = np.abs(sym.astype(np.float32))
    n = 2 * np.floor(np.log2(s / np.float32(2 ** count) + 1)) + count + 1 + (sym != 0)
    return float(n.sum())


def best_count(sym: np.ndarray) -> tuple[int, float]:
    best, rate = 0, None
    for c in EXPGOL_COUNTS:
        r = exp_golomb_nbins(sym, int(c))
        if rate is None or r < rate:
            best, rate = int(c), r
    return best, rate


@dataclass
class Layout:
    """Index ranges of the parameter block (ccmi.train layout) per module and kind."""
    arm_w: np.ndarray
    arm_b: np.ndarray
    ups_w: np.ndarray
    syn_w: np.ndarray
    syn_b: np.ndarray
    syn_off: int
    P: int

    @classmethod
    def of(cls, a: Arch) -> "Layout":
        d, p = a.dim_arm, 0
        aw, ab = [], []
        for l in range(a.n_hidden + 1):
            n_out = d if l < a.n_hidden else 2
            aw += range(p, p + n_out * d)
            p += n_out * d
            ab += range(p, p + n_out)
            p += n_out
        hu, hp = (a.ups_k + 1) // 2, (a.pre_k + 1) // 2
        uw = list(range(p, p + (a.n_grids - 1) * (hu + hp)))
        p += (a.n_grids - 1) * (hu + hp)
        syn_off = p
        sw, sb, c = [], [], a.n_grids
        for n_out, k, _, _ in a.layers:
            sw += range(p, p + n_out * c * k * k)
            p += n_out * c * k * k
            sb += range(p, p + n_out)
            p += n_out
            c = n_out
        A = lambda x: np.asarray(x, dtype=np.int64)  # noqa: E731
        return cls(A(aw), A(ab), A(uw), A(sw), A(sb), syn_off, p)

    def kinds(self, module: str):
        return {"arm": (self.arm_w, self.arm_b), "upsampling": (self.ups_w, None),
                "synthesis": (self.syn_w, self.syn_b)}[module]


@dataclass
class QuantizedModel:
    params: np.ndarray                         # float32 quantised parameter block
    q_index: dict = field(default_factory=dict)  # module -> (weight index, bias index)
    q_step: dict = field(default_factory=dict)   # module -> (weight step, bias step)
    expgol: dict = field(default_factory=dict)   # module -> (weight count, bias count)
    nn_bits: dict = field(default_factory=dict)  # module -> Exp-Golomb bits of its weights + biases
    loss: float = 0.0
    # module -> [(q_w, q_b, loss)] for every candidate tried, in the reference's order; the loss
    # omits the terms that are the same for every candidate of that module (module docstring)
    table: dict = field(default_factory=dict)


def _full_kernels(arch: Arch, blocks: torch.Tensor, lay: Layout) -> torch.Tensor:
    """Half kernels of each candidate block -> full symmetric kernels (ccmi_ups_args order)."""
    hu, hp = (arch.ups_k + 1) // 2, (arch.pre_k + 1) // 2
    u = blocks[:, lay.ups_w]
    out = []
    for i in range(arch.n_grids - 1):
        h = u[:, i * hu:(i + 1) * hu]
        out.append(torch.cat([h, torch.flip(h, [1])[:, arch.ups_k % 2:]], dim=1))
    base = (arch.n_grids - 1) * hu
    for i in range(arch.n_grids - 1):
        h = u[:, base + i * hp: base + (i + 1) * hp]
        out.append(torch.cat([h, torch.flip(h, [1])[:, arch.pre_k % 2:]], dim=1))
    return torch.cat(out, dim=1).contiguous()


class _Eval:
    """Batched eval forwards with shared latents / shared stages (stride-0 inputs)."""

    def __init__(self, arch: Arch, latent: torch.Tensor, target: torch.Tensor, yuv420: bool, bitdepth: int):
        self.a, self.lat, self.tgt, self.yuv420, self.bd = arch, latent.contiguous(), target.contiguous(), yuv420, bitdepth
        self.dev = latent.device
        self.h = (C.c_int * MAX_GRIDS)(*[s[0] for s in arch.sizes])
        self.w = (C.c_int * MAX_GRIDS)(*[s[1] for s in arch.sizes])
        self.L = lib()
        self.L.ccmi_row_reduce_f32.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int,
                                               C.c_int, C.c_void_p, C.c_void_p]
        self.L.ccmi_row_reduce_f32.restype = C.c_int
        self.s = torch.cuda.current_stream(self.dev).cuda_stream

    def reduce(self, a: torch.Tensor, t: torch.Tensor | None, mode: int) -> torch.Tensor:
        B = a.shape[0]
        out = torch.empty(B, dtype=torch.float64, device=self.dev)
        check(self.L.ccmi_row_reduce_f32(a.data_ptr(), a.shape[1], None if t is None else t.data_ptr(),
                                         0 if t is None or t.dim() == 1 else t.shape[1], a.shape[1], B, mode,
                                         out.data_ptr(), self.s))
        return out

    def rate_sum(self, blocks: torch.Tensor) -> torch.Tensor:
        """ARM + Laplace rate (bits) of the shared latents, one row per candidate block."""
        a = self.a
        B, N = blocks.shape[0], a.n_latents
        rate = torch.empty(B, N, device=self.dev)
        args = ArmArgs(latent=self.lat.data_ptr(), latent_stride=0, n_grids=a.n_grids, h=self.h, w=self.w,
                       gain=a.gain, quantize=1, dim_arm=a.dim_arm, n_hidden=a.n_hidden, params=blocks.data_ptr(),
                       param_stride=blocks.shape[1], mu=None, scale=None, log_scale=None, rate=rate.data_ptr(),
                       out_stride=N, batch=B)
        check(self.L.ccmi_arm_forward_f32(C.byref(args), self.s))
        return self.reduce(rate, None, 0)

    def dense(self, kernels: torch.Tensor, shared_latent: bool = True) -> torch.Tensor:
        a = self.a
        B = kernels.shape[0]
        H, W = a.sizes[0]
        out = torch.empty(B, a.n_grids, H, W, device=self.dev)
        nws = self.L.ccmi_ups_workspace_bytes(a.n_grids, self.h, self.w, B)
        ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=self.dev)
        args = UpsArgs(latent=self.lat.data_ptr(), latent_stride=0, n_grids=a.n_grids, h=self.h, w=self.w,
                       gain=a.gain, quantize=1, ups_k=a.ups_k, n_ups=a.n_grids - 1, pre_k=a.pre_k,
                       n_pre=a.n_grids - 1, params=kernels.data_ptr(), param_stride=kernels.shape[1],
                       out=out.data_ptr(), out_stride=a.n_grids * H * W, workspace=ws.data_ptr(),
                       workspace_bytes=nws, batch=B)
        check(self.L.ccmi_ups_forward_f32(C.byref(args), self.s))
        return out

    def mse(self, dense: torch.Tensor, syn: torch.Tensor) -> torch.Tensor:
        """Synthesis + eval post-processing + MSE vs the target; dense [1 or B] (stride 0
        when shared), syn [1 or B] parameter rows."""
        a = self.a
        B = max(dense.shape[0], syn.shape[0])
        H, W = a.sizes[0]
        raw = torch.empty(B, 3, H, W, device=self.dev)
        arr = (SynLayer * MAX_SYN_LAYERS)()
        for i, (n, k, r, nl) in enumerate(a.layers):
            arr[i] = SynLayer(int(n), int(k), int(r), int(nl))
        sa = SynArgs(in_=dense.data_ptr(), in_stride=0 if dense.shape[0] == 1 else a.n_grids * H * W,
                     c_in=a.n_grids, h=H, w=W, n_layers=len(a.layers), layers=arr, params=syn.data_ptr(),
                     param_stride=0 if syn.shape[0] == 1 else syn.shape[1], out=raw.data_ptr(), out_stride=3 * H * W,
                     workspace=None, workspace_bytes=0, batch=B)
        nws = self.L.ccmi_syn_workspace_bytes(C.byref(sa))
        if nws:
            ws = torch.empty(nws, dtype=torch.uint8, device=self.dev)
            sa.workspace, sa.workspace_bytes = ws.data_ptr(), nws
        check(self.L.ccmi_syn_forward_f32(C.byref(sa), self.s))
        n = H * W + 2 * (H // 2) * (W // 2) if self.yuv420 else 3 * H * W
        dec = torch.empty(B, n, device=self.dev)
        pa = PostArgs(in_=raw.data_ptr(), in_stride=3 * H * W, h=H, w=W, bitdepth=self.bd, yuv420=int(self.yuv420),
                      out=dec.data_ptr(), out_stride=n, batch=B)
        check(self.L.ccmi_post_f32(C.byref(pa), self.s))
        return self.reduce(dec, self.tgt, 1) / n


def quantize_model(arch: Arch, latent: torch.Tensor, params: torch.Tensor, target: torch.Tensor, lmbda: float,
                   yuv420: bool = True, bitdepth: int = 8, chunk: int = 64) -> QuantizedModel:
    """Greedy per-module search of the quantisation steps (quantizemodel.py:120-245) for
    one frame: latent [N] (float, before gain), params [P] (ccmi.train layout), target
    (flat, ccmi.train layout) on the GPU."""
    lay = Layout.of(arch)
    ev = _Eval(arch, latent.float(), target.float(), yuv420, bitdepth)
    fp = params.detach().float().cpu().numpy()
    cur = fp.copy()
    res = QuantizedModel(params=cur)
    H, W = arch.sizes[0]
    npx = H * W
    for module in ("arm", "synthesis", "upsampling"):
        wi, bi = lay.kinds(module)
        cands, blocks, nn_rate, counts = [], [], [], []
        for iw, qw in enumerate(POSSIBLE_Q_STEP[module]["weight"]):
            for ib, qb in enumerate(POSSIBLE_Q_STEP[module]["bias"]):
                qw32, qb32 = np.float32(qw), np.float32(qb)
                sw = np.round(fp[wi] / qw32)
                if np.abs(sw).max(initial=0) > MAX_AC_MAX_VAL:
                    continue
                b = cur.copy()
                b[wi] = sw * qw32
                cw, rw = best_count(sw)
                cb, rb = 0, 0.0
                if bi is not None:
                    sb = np.round(fp[bi] / qb32)
                    if np.abs(sb).max(initial=0) > MAX_AC_MAX_VAL:
                        continue
                    b[bi] = sb * qb32
                    cb, rb = best_count(sb)
                cands.append((iw, ib, float(qw), float(qb)))
                blocks.append(b)
                nn_rate.append(rw + rb)
                counts.append((cw, cb))
        if not cands:
            raise RuntimeError(f"quantize_model: no valid quantisation step for {module}")
        losses = []
        base_dense = None
        for s0 in range(0, len(blocks), chunk):
            blk = torch.from_numpy(np.stack(blocks[s0:s0 + chunk])).to(ev.dev)
            if module == "arm":
                part = lmbda * ev.rate_sum(blk) / npx
            elif module == "synthesis":
                if base_dense is None:
                    base_dense = ev.dense(_full_kernels(arch, torch.from_numpy(cur)[None].to(ev.dev), lay))
                part = ev.mse(base_dense, blk[:, lay.syn_off:].contiguous())
            else:
                dense = ev.dense(_full_kernels(arch, blk, lay))
                part = ev.mse(dense, torch.from_numpy(cur[lay.syn_off:])[None].to(ev.dev).contiguous())
            losses.append(part.cpu())
        loss = torch.cat(losses).numpy() + lmbda * np.asarray(nn_rate) / npx
        k = int(np.argmin(loss))  # first minimum, as the reference's strict "<"
        iw, ib, qw, qb = cands[k]
        cur = blocks[k]
        res.q_index[module] = (iw, ib)
        res.q_step[module] = (qw, qb)
        res.expgol[module] = counts[k]
        res.nn_bits[module] = float(nn_rate[k])
        res.loss = float(loss[k])
        res.table[module] = [(c[2], c[3], float(v)) for c, v in zip(cands, loss)]
    res.params = cur
    return res


def evaluate(arch: Arch, latent: torch.Tensor, params: torch.Tensor, target: torch.Tensor, yuv420: bool = True,
             bitdepth: int = 8) -> tuple[float, float]:
    """test() of enc/training/test.py:370-438 for one frame, on the GPU: MSE of the eval
    forward (hard-rounded latents, output on the 2^bitdepth - 1 grid, 420 subsampling) and
    the latent rate in bits.  The network rate of a quantised model is
    QuantizedModel.nn_bits."""
    lay = Layout.of(arch)
    ev = _Eval(arch, latent.float(), target.float(), yuv420, bitdepth)
    p = params.detach().float().reshape(1, -1).to(ev.dev).contiguous()
    rate = float(ev.rate_sum(p)[0])
    dense = ev.dense(_full_kernels(arch, p, lay))
    mse = float(ev.mse(dense, p[:, lay.syn_off:].contiguous())[0])
    return mse, rate


__all__ = ["quantize_model", "QuantizedModel", "Layout", "POSSIBLE_Q_STEP", "exp_golomb_nbins", "best_count",
           "evaluate"]
