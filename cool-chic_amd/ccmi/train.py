"""Encoder overfit step on the GPU (ccmi_train_step): the training forward, backward,
clip_grad_norm_ and Adam of enc/training/train.py:238-262, for a batch of independent
frames.  Torch tensors are storage only; every FLOP runs in libccmi's HIP kernels.

Parameter block per frame (float32), in this order:
  ARM      per hidden layer W [d][d] (out, in) then b [d]; W_out [2][d], b_out [2]
           (arm.mlp state_dict order, arm.py:86-101);
  UPS      n_ups half kernels of (ups_k + 1) // 2 taps
           (upsampling.conv_transpose2ds.{i}.parametrizations.weight.original);
  PRE      n_pre half kernels of (pre_k + 1) // 2 taps
           (upsampling.conv2ds.{i}.parametrizations.weight.original);
  SYN      per layer W [n_out][c_in][k][k] then b [n_out] (synthesis.layers.{2i}).
"""

from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Sequence

import torch

from . import MAX_GRIDS, MAX_SYN_LAYERS, SynLayer, check, lib, require_cuda

Q_TYPES = {"none": 0, "softround_alone": 1, "softround": 2, "hardround": 3, "ste": 4, "true_ste": 5}
NOISE_TYPES = {"none": 0, "kumaraswamy": 1, "gaussian": 2}


class TrainArgs(C.Structure):
    _fields_ = [
        ("batch", C.c_int), ("n_grids", C.c_int), ("h", C.c_int * MAX_GRIDS), ("w", C.c_int * MAX_GRIDS),
        ("dim_arm", C.c_int), ("n_hidden", C.c_int), ("ups_k", C.c_int), ("n_ups", C.c_int), ("pre_k", C.c_int),
        ("n_pre", C.c_int), ("n_syn_layers", C.c_int), ("syn", SynLayer * MAX_SYN_LAYERS), ("gain", C.c_float),
        ("latent", C.c_void_p), ("latent_stride", C.c_int64), ("params", C.c_void_p), ("param_stride", C.c_int64),
        ("adam_m", C.c_void_p), ("adam_v", C.c_void_p), ("target", C.c_void_p), ("target_stride", C.c_int64),
        ("yuv420", C.c_int), ("quantizer", C.c_int), ("noise", C.c_int), ("temperature", C.c_float),
        ("noise_param", C.c_float), ("lmbda", C.c_float), ("lr", C.c_float), ("beta1", C.c_float),
        ("beta2", C.c_float), ("eps", C.c_float), ("clip", C.c_float), ("step", C.c_int), ("seed", C.c_uint64),
        ("noise_in", C.c_void_p), ("grad_out", C.c_void_p), ("loss_out", C.c_void_p), ("update", C.c_int),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
        ("forward_only", C.c_int), ("raw_out", C.c_void_p), ("rate_out", C.c_void_p), ("grad_raw", C.c_void_p),
        ("grad_rate", C.c_void_p), ("adam_steps", C.c_void_p), ("step_counters", C.c_void_p),
    ]


def _bind():
    L = lib()
    if not getattr(L, "_ccmi_train_bound", False):
        L.ccmi_train_step.argtypes = [C.POINTER(TrainArgs), C.c_void_p]
        L.ccmi_train_step.restype = C.c_int
        L.ccmi_train_workspace_bytes.argtypes = [C.POINTER(TrainArgs)]
        L.ccmi_train_workspace_bytes.restype = C.c_size_t
        L.ccmi_train_param_count.argtypes = [C.POINTER(TrainArgs)]
        L.ccmi_train_param_count.restype = C.c_size_t
        L._ccmi_train_bound = True
    return L


@dataclass
class Arch:
    H: int
    W: int
    dim_arm: int = 16
    n_hidden: int = 2
    layers: tuple = ((48, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False))
    n_grids: int = 7
    ups_k: int = 8
    pre_k: int = 7
    gain: float = 16.0

    @property
    def sizes(self):
        s, h, w = [], self.H, self.W
        for _ in range(self.n_grids):
            s.append((h, w))
            h, w = (h + 1) // 2, (w + 1) // 2
        return s

    @property
    def n_latents(self) -> int:
        return sum(h * w for h, w in self.sizes)


def init_params(arch: Arch, generator: torch.Generator | None = None) -> torch.Tensor:
    """Parameter block of a freshly constructed CoolChicEncoder: ARM residual layers zero,
    output layer N(0, 1/C_out^4) (arm.py:66-84); upsampling bicubic / bilinear half kernels
    (upsampling.py:262-292) and Dirac refine kernels (:131-150); synthesis residual layers
    zero, others U(-a, a), a = 1 / (C_out^2 sqrt(C_in k^2)) (synthesis.py:86-116); biases 0."""
    g = generator or torch.Generator().manual_seed(0)
    d = arch.dim_arm
    arm = [(torch.zeros(d, d), torch.zeros(d)) for _ in range(arch.n_hidden)]
    arm.append((torch.randn(2, d, generator=g) / 2 ** 2, torch.zeros(2)))
    hu, hp = (arch.ups_k + 1) // 2, (arch.pre_k + 1) // 2
    core = torch.tensor([1.0 / 4.0, 3.0 / 4.0]) if arch.ups_k < 8 else \
        torch.tensor([0.0351562, 0.1054687, -0.2617187, -0.8789063])
    up = torch.zeros(hu)
    up[hu - core.numel():] = core
    pre = torch.zeros(hp)
    pre[-1] = 1.0
    syn, c = [], arch.n_grids
    for n_out, k, res, _ in arch.layers:
        if res:
            W = torch.zeros(n_out, c, k, k)
        else:
            a = math.sqrt(1.0 / (c * k * k)) / n_out ** 2
            W = (torch.rand(n_out, c, k, k, generator=g) - 0.5) * 2 * a
        syn.append((W, torch.zeros(n_out)))
        c = n_out
    return pack_params(arm, [up] * (arch.n_grids - 1), [pre] * (arch.n_grids - 1), syn)


def pack_params(arm, ups_half, pre_half, syn) -> torch.Tensor:
    """[(W, b)...], [half...], [half...], [(W, b)...] -> flat float32 parameter block."""
    parts = [t.reshape(-1).float() for wb in arm for t in wb]
    parts += [h.reshape(-1).float() for h in list(ups_half) + list(pre_half)]
    parts += [t.reshape(-1).float() for wb in syn for t in wb]
    return torch.cat(parts)


class Overfitter:
    """GPU state of `batch` frames being overfitted together: latents, parameters and the
    Adam moments live in HBM; step() runs one training iteration for all of them."""

    def __init__(self, arch: Arch, latents: torch.Tensor, params: torch.Tensor, targets: torch.Tensor,
                 yuv420: bool = True, seed: int = 0):
        require_cuda(latents, params, targets)
        self.arch, self.yuv420, self.seed = arch, bool(yuv420), seed
        self.B = latents.shape[0]
        self.latents = latents.float().contiguous()
        self.params = params.float().contiguous()
        self.targets = targets.float().contiguous()
        self.t = 0
        a = self._args()
        L = _bind()
        P = L.ccmi_train_param_count(C.byref(a))
        if P == 0 or self.params.shape[1] != P:
            raise ValueError(f"params: expected [B, {P}] for this architecture, got {tuple(self.params.shape)}")
        if self.latents.shape[1] != arch.n_latents:
            raise ValueError(f"latents: expected [B, {arch.n_latents}]")
        self.P, self.N = P, arch.n_latents
        dev = self.latents.device
        self.m = torch.zeros(self.B, self.N + P, device=dev)
        self.v = torch.zeros(self.B, self.N + P, device=dev)
        # each frame's Adam step (frames diverge when one reloads its best optimizer state,
        # train.py:226-236); uniform steps use the scalar path
        self.steps = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.steps_uniform = True
        self.loss = torch.zeros(self.B, 4, device=dev)
        self.ws = torch.empty(L.ccmi_train_workspace_bytes(C.byref(a)), dtype=torch.uint8, device=dev)

    def reset_optimizer(self):
        """A new torch.optim.Adam: every training phase builds its own (train.py:184)."""
        self.m.zero_()
        self.v.zero_()
        self.steps.zero_()
        self.steps_uniform = True
        self.t = 0

    def _realloc(self):
        self.loss = torch.zeros(self.B, 4, device=self.latents.device)
        a = self._args()
        self.ws = torch.empty(_bind().ccmi_train_workspace_bytes(C.byref(a)), dtype=torch.uint8,
                              device=self.latents.device)

    def keep(self, idx: torch.Tensor):
        """Keep frames idx (a [B'] index tensor) of the batch, in that order."""
        idx = idx.to(self.latents.device)
        self.latents = self.latents[idx].contiguous()
        self.params = self.params[idx].contiguous()
        self.targets = self.targets[idx].contiguous()
        self.m, self.v = self.m[idx].contiguous(), self.v[idx].contiguous()
        self.steps = self.steps[idx].contiguous()
        self.B = int(idx.numel())
        self._realloc()

    def reset_batch(self, latents: torch.Tensor, params: torch.Tensor, targets: torch.Tensor):
        """Replace the batch (fresh optimizer state)."""
        self.latents, self.params = latents.float().contiguous(), params.float().contiguous()
        self.targets = targets.float().contiguous()
        self.B = self.latents.shape[0]
        dev = self.latents.device
        self.m = torch.zeros(self.B, self.N + self.P, device=dev)
        self.v = torch.zeros(self.B, self.N + self.P, device=dev)
        self.steps = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.steps_uniform = True
        self.t = 0
        self._realloc()

    def validate(self, lmbda: float) -> torch.Tensor:
        """Loss of the hard-rounded forward (train.py test(): quantizer "hardround", no
        noise), without the eval-mode 8-bit rounding of the decoded image."""
        return self.step("hardround", "none", 1.0, 1.0, lmbda, update=False).clone()

    def _args(self) -> TrainArgs:
        ar = self.arch
        a = TrainArgs()
        a.batch, a.n_grids = self.B, ar.n_grids
        for i, (h, w) in enumerate(ar.sizes):
            a.h[i], a.w[i] = h, w
        a.dim_arm, a.n_hidden = ar.dim_arm, ar.n_hidden
        a.ups_k, a.n_ups, a.pre_k, a.n_pre = ar.ups_k, ar.n_grids - 1, ar.pre_k, ar.n_grids - 1
        a.n_syn_layers = len(ar.layers)
        for i, (n, k, r, nl) in enumerate(ar.layers):
            a.syn[i] = SynLayer(n, k, int(r), int(nl))
        a.gain = ar.gain
        a.latent, a.latent_stride = self.latents.data_ptr(), self.latents.shape[1]
        a.params, a.param_stride = self.params.data_ptr(), self.params.shape[1]
        a.target, a.target_stride = self.targets.data_ptr(), self.targets.shape[1]
        a.yuv420 = int(self.yuv420)
        return a

    def step(self, quantizer_type="softround", quantizer_noise_type="kumaraswamy", soft_round_temperature=0.3,
             noise_parameter=1.0, lmbda=1e-3, lr=1e-2, clip=0.1, update=True, noise=None, grad_out=None):
        """One iteration; returns [B, 4] (loss, mse, rate_bits, grad_norm) of this step's forward.
        update: False (gradients only), True / "all" (Adam on everything), "latent"."""
        a = self._args()
        if update:
            self.t += 1
            a.step_counters = self.steps.data_ptr()  # self.steps += 1, inside the step's prologue
            if not self.steps_uniform:
                a.adam_steps = self.steps.data_ptr()
        a.adam_m, a.adam_v = self.m.data_ptr(), self.v.data_ptr()
        a.quantizer, a.noise = Q_TYPES[quantizer_type], NOISE_TYPES[quantizer_noise_type]
        a.temperature, a.noise_param, a.lmbda = float(soft_round_temperature), float(noise_parameter), float(lmbda)
        a.lr, a.beta1, a.beta2, a.eps, a.clip = float(lr), 0.9, 0.999, 1e-8, float(clip)
        a.step = max(self.t, 1)
        a.seed = self.seed
        if noise is not None:
            require_cuda(noise)
            noise = noise.float().contiguous()
            a.noise_in = noise.data_ptr()
        if grad_out is not None:
            if grad_out.shape != (self.B, self.N + self.P) or not grad_out.is_contiguous():
                raise ValueError("grad_out: contiguous [B, N + P] expected")
            a.grad_out = grad_out.data_ptr()
        a.loss_out = self.loss.data_ptr()
        a.update = 2 if update == "latent" else int(bool(update))
        a.workspace, a.workspace_bytes = self.ws.data_ptr(), self.ws.numel()
        check(_bind().ccmi_train_step(C.byref(a), torch.cuda.current_stream(self.latents.device).cuda_stream))
        return self.loss


def cosine_lr(start: float, end: float, it: int, max_it: int, freq: int) -> float:
    """CosineAnnealingLR(T_max = max_itr / freq_valid, eta_min = end) stepped every freq
    iterations (train.py:189-196, :351-352)."""
    T = max_it / freq
    e = it // freq
    return end + (start - end) * (1 + math.cos(math.pi * e / T)) / 2


def linear(a: float, b: float, it: int, max_it: int) -> float:
    """_linear_schedule (train.py)."""
    return a + (b - a) * it / max_it


@dataclass
class Phase:
    """TrainerPhase (enc/training/presets.py:25-110)."""
    lr: float = 1e-2
    max_itr: int = 5000
    freq_valid: int = 100
    patience: int = 10000
    schedule_lr: bool = False
    end_lr: float = 1e-5
    softround_temperature: tuple = (0.3, 0.3)
    noise_parameter: tuple = (1.0, 1.0)
    quantizer_noise_type: str = "kumaraswamy"
    quantizer_type: str = "softround"
    optimized_module: str = "all"
    quantize_model: bool = False


# preset_cfg/c3x.yaml
C3X_WARMUP = [(5, Phase(lr=1e-2, max_itr=400, freq_valid=400, patience=100000, noise_parameter=(2.0, 2.0))),
              (2, Phase(lr=1e-2, max_itr=400, freq_valid=400, patience=100000, noise_parameter=(2.0, 2.0)))]
C3X_PHASES = [
    Phase(lr=1e-2, max_itr=10600, patience=5000, schedule_lr=True, quantizer_noise_type="gaussian",
          softround_temperature=(0.3, 0.1), noise_parameter=(0.25, 0.1)),
    Phase(lr=1e-4, max_itr=1500, patience=1500, schedule_lr=True, quantizer_type="ste", quantizer_noise_type="none",
          softround_temperature=(1e-4, 1e-4), quantize_model=True),
    Phase(lr=1e-4, max_itr=1000, patience=50, quantizer_type="ste", quantizer_noise_type="none",
          optimized_module="latent", freq_valid=10, softround_temperature=(1e-4, 1e-4)),
]


# preset "debug" (preset_cfg/debug.yaml, the file the reference's encoder loads with --preset and
# tools/gen_golden_rd.py ran the R-D fixtures from): the schedule of the reference's sanity check.
# Its warm-up trains with kumaraswamy noise parameter 2.0, freq_valid 400, patience 100000 -- the
# legacy class enc/training/presets.py:380-432 (PresetDebug) leaves the TrainerPhase defaults
# (noise 1.0), which this schedule followed until round 6.
DEBUG_WARMUP = [(3, Phase(lr=1e-2, max_itr=10, freq_valid=400, patience=100000, noise_parameter=(2.0, 2.0))),
                (2, Phase(lr=1e-2, max_itr=10, freq_valid=400, patience=100000, noise_parameter=(2.0, 2.0)))]
DEBUG_PHASES = [
    Phase(lr=1e-2, max_itr=50, patience=100000, schedule_lr=True, quantizer_noise_type="gaussian",
          softround_temperature=(0.3, 0.1), noise_parameter=(0.25, 0.1)),
    Phase(lr=1e-4, max_itr=10, patience=10, quantizer_type="ste", quantizer_noise_type="none", quantize_model=True,
          softround_temperature=(1e-4, 1e-4)),
    Phase(lr=1e-4, max_itr=10, patience=50, optimized_module="latent", freq_valid=5, quantizer_type="ste",
          quantizer_noise_type="none", softround_temperature=(1e-4, 1e-4)),
]


def c3x_iterations(scale: float = 1.0) -> int:
    """Training iterations per image of the c3x preset (x scale): warm-up candidates
    trained in parallel count once per surviving image."""
    return sum(max(1, int(p.max_itr * scale)) for _, p in C3X_WARMUP) + \
        sum(max(1, int(p.max_itr * scale)) for p in C3X_PHASES)


def run_phase(of: Overfitter, ph: Phase, lmbda: float, scale: float = 1.0) -> torch.Tensor:
    """train() (enc/training/train.py:86-374) for every frame of the batch at once: Adam
    restarted, cosine learning rate stepped every freq_valid iterations, linear soft-round
    temperature / noise schedules, validation every freq_valid iterations keeping each
    frame's best parameters (restored at the end of the phase).  A validation is a new
    record when its loss is lower AND it gains more than 0.001 dB or loses less than
    0.001 bpp (train.py:280-289).

    Patience, per frame, as train.py:226-240: at the start of iteration cnt, a frame whose
    last record is more than `patience` iterations old either reloads its best parameters
    and Adam state (cosine-scheduled phases; the learning rate stays the schedule's) or
    stops (other phases: it leaves the batch, so the remaining frames run alone).  With
    scale < 1, patience and freq_valid are scaled like max_itr (as tools/gen_golden_rd.py
    scales the reference's presets).  Sets of.phase_iterations (per frame of the batch, in
    batch order).  Returns the best validation [B, 4]."""
    n = max(1, int(ph.max_itr * scale))
    freq = max(1, int(ph.freq_valid * scale)) if scale < 1 else ph.freq_valid
    pat = max(1, int(ph.patience * scale)) if scale < 1 else ph.patience
    npx = of.arch.sizes[0][0] * of.arch.sizes[0][1]
    B0 = of.B
    dev = of.latents.device
    of.reset_optimizer()
    best = of.validate(lmbda).clone()
    best_lat, best_prm = of.latents.clone(), of.params.clone()
    # reload targets: Adam moments and steps at the record (cosine phases only)
    reload = ph.schedule_lr and pat < n
    if reload:
        best_m, best_v, best_st = of.m.clone(), of.v.clone(), of.steps.clone()
    full_tg = of.targets
    rows = list(range(B0))                   # frame (original batch index) of each row of `of`
    rec = [0] * B0                           # cnt_record per frame
    its = [0] * B0
    T = ph.softround_temperature[0]
    nz = ph.noise_parameter[0]
    upd = "latent" if ph.optimized_module == "latent" else True
    for cnt in range(n):
        late = [r for r, f in enumerate(rows) if cnt - rec[f] > pat]
        if late:
            if reload:
                ri = torch.tensor(late, device=dev)
                fi = torch.tensor([rows[r] for r in late], device=dev)
                of.latents[ri] = best_lat[fi]
                of.params[ri] = best_prm[fi]
                of.m[ri] = best_m[fi]
                of.v[ri] = best_v[fi]
                of.steps[ri] = best_st[fi]
                of.steps_uniform = False
                for r in late:
                    rec[rows[r]] = cnt
            else:
                keep = [r for r in range(len(rows)) if r not in late]
                if not keep:
                    break
                of.keep(torch.tensor(keep, device=dev))
                rows = [rows[r] for r in keep]
        lr = cosine_lr(ph.lr, ph.end_lr, cnt, n, freq) if ph.schedule_lr else ph.lr
        of.step(ph.quantizer_type, ph.quantizer_noise_type, T, nz, lmbda, lr=lr, update=upd)
        for f in rows:
            its[f] += 1
        if (cnt + 1) % freq == 0 or cnt + 1 == n:
            cur = of.validate(lmbda)
            fi = torch.tensor(rows, device=dev)
            bst = best[fi]
            d_psnr = 10 * torch.log10(bst[:, 1].clamp_min(1e-10) / cur[:, 1].clamp_min(1e-10))
            d_bpp = (cur[:, 2] - bst[:, 2]) / npx
            better = (cur[:, 0] < bst[:, 0]) & ((d_bpp < 1e-3) | (d_psnr > 1e-3))
            bl = better.tolist()
            if any(bl):
                ri = torch.tensor([r for r, v in enumerate(bl) if v], device=dev)
                fb = fi[ri]
                best[fb] = cur[ri]
                best_lat[fb] = of.latents[ri]
                best_prm[fb] = of.params[ri]
                if reload:
                    best_m[fb] = of.m[ri]
                    best_v[fb] = of.v[ri]
                    best_st[fb] = of.steps[ri]
                for r, v in enumerate(bl):
                    if v:
                        rec[rows[r]] = cnt
            T = linear(ph.softround_temperature[0], ph.softround_temperature[1], cnt, n)
            nz = linear(ph.noise_parameter[0], ph.noise_parameter[1], cnt, n)
    # every frame ends on its best record (train.py:372-373)
    if len(rows) == B0:
        of.latents.copy_(best_lat)
        of.params.copy_(best_prm)
    else:
        of.reset_batch(best_lat, best_prm, full_tg)
    of.phase_iterations = its
    return best


def overfit(arch: Arch, targets: torch.Tensor, lmbda: float, yuv420: bool = True, scale: float = 1.0,
            seed: int = 0, warmup=C3X_WARMUP, phases=C3X_PHASES, bitdepth: int = 8) -> tuple[Overfitter, torch.Tensor]:
    """The c3x encoding schedule (enc/training/warmup.py + train.py phases) for a batch of
    frames [B, target_len] on one GPU.  Warm-up candidates of every frame train together
    as one batch; after each warm-up stage each frame keeps its best candidates.  After a
    phase flagged quantize_model, every frame's networks are quantised
    (ccmi.quantize.quantize_model, as video.py:302-310) and later phases train with them;
    the per-frame QuantizedModel list is state.quantized (None if no phase asks for it);
    state.iterations the per-frame iteration counts.  Returns (state, best validation)."""
    import time
    dev = targets.device
    B = targets.shape[0]
    n0 = warmup[0][0] if warmup else 1
    stream = torch.cuda.current_stream(dev)
    timing = {"warmup_s": 0.0, "phases_s": [], "quantize_s": 0.0}
    t0 = time.perf_counter()
    g = torch.Generator().manual_seed(seed)
    params = torch.stack([init_params(arch, g) for _ in range(B * n0)]).to(dev)
    lat = torch.zeros(B * n0, arch.n_latents, device=dev)
    of = Overfitter(arch, lat, params, targets.repeat_interleave(n0, dim=0), yuv420=yuv420, seed=seed)
    ncand = n0
    # iterations per image as the reference's FrameEncoderManager.iterations_counter counts
    # them: the sum over the image's own warm-up candidates (trained one after another in
    # warmup.py), then the phases' (early stops included).  Rows of `of` are image-major.
    warm_its = [0] * B
    for i, (_, ph) in enumerate(warmup):
        res = run_phase(of, ph, lmbda, scale)
        for b in range(B):
            warm_its[b] += sum(of.phase_iterations[b * ncand:(b + 1) * ncand])
        keep = warmup[i + 1][0] if i + 1 < len(warmup) else 1
        order = torch.argsort(res[:, 0].view(B, ncand), dim=1)[:, :keep]
        idx = (order + torch.arange(B, device=order.device)[:, None] * ncand).reshape(-1)
        of.keep(idx)
        ncand = keep
    best = None
    of.quantized = None
    of.iterations = list(warm_its)
    stream.synchronize()
    timing["warmup_s"] = time.perf_counter() - t0
    for ph in phases:
        t0 = time.perf_counter()
        best = run_phase(of, ph, lmbda, scale)
        of.iterations = [a + b for a, b in zip(of.iterations, of.phase_iterations)]
        stream.synchronize()
        timing["phases_s"].append(time.perf_counter() - t0)
        if ph.quantize_model:
            from .quantize import quantize_model
            t0 = time.perf_counter()
            qms = []
            for b in range(of.B):
                qm = quantize_model(arch, of.latents[b], of.params[b], of.targets[b], lmbda, yuv420, bitdepth)
                of.params[b].copy_(torch.from_numpy(qm.params).to(of.params.device))
                qms.append(qm)
            of.quantized = qms
            best = of.validate(lmbda).clone()
            stream.synchronize()
            timing["quantize_s"] += time.perf_counter() - t0
    # wall seconds of the schedule's parts (host clock, this stream synchronised at each
    # boundary): what the bench's encoder leg reports next to its images/hr
    of.timing = timing
    return of, best


__all__ = ["Arch", "Overfitter", "Phase", "C3X_WARMUP", "C3X_PHASES", "DEBUG_WARMUP", "DEBUG_PHASES", "c3x_iterations", "run_phase", "overfit",
           "init_params", "pack_params", "cosine_lr", "linear", "Q_TYPES", "NOISE_TYPES"]
