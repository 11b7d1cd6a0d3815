"""Kernel orchestration for one PointNetSegmentation training / inference pass.

Host side of the hot path: allocates (through torch's caching allocator) the points-major
activation buffers, and launches the HIP kernels of libpcs.so in dependency order on the
current stream.  Nothing here computes on the CPU; every numeric op is a C-ABI call.

Per layer l the forward stores only Y_l = conv_l(a_{l-1}) (pre-BN, fp32 or bf16);
a_l = relu(bn_l(Y_l)) [* dropout] is recomputed inside whichever kernel consumes it.
The exception is the 1024-wide pair conv5 / global_feat: conv5 runs twice (a statistics pass,
then a pass that applies bn5 + ReLU on the way out), so a5 = relu(bn5(y5)) is stored instead of
y5, and global_feat's output is never stored (its epilogue keeps only BN statistics and the
max-pool candidates).  Both 1024-deep global_feat GEMMs then read a5 raw, which lets them stage
it HBM -> LDS by DMA (csrc/gemm_glds.hip).
The backward stores dZ_l = dL/d(BN_l output) after the ReLU / dropout masks and forms
dy_l = alpha*dZ_l + beta + gamma*Y_l on the fly in the dgrad / wgrad kernels.

Reference map (point_cloud_segmentation.py, P:<line>):
  forward P:98-133, loss P:216/251, backward P:254, running stats (nn.BatchNorm1d).
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass, field

import torch

from . import _lib as L

BN_EPS = 1e-5
MAX_INPUT_DIM = 8     # conv1 kernels (csrc/small.hip) are instantiated for K = 1..8
MAX_CLASSES = 256     # head kernels (csrc/small.hip: 16 / 64 classes, and the wide head up to 256)
BN_MOMENTUM = 0.1
DROPOUT_P = 0.3

# (conv, Cin, Cout, bn) in registration order; Cin of conv1 / Cout of seg_conv4 filled in
CONVS = [
    ("conv1", None, 64, "bn1"),
    ("conv2", 64, 64, "bn2"),
    ("conv3", 64, 64, "bn3"),
    ("conv4", 64, 128, "bn4"),
    ("conv5", 128, 1024, "bn5"),
    ("global_feat", 1024, 1024, "bn_global"),
    ("seg_conv1", 1088, 512, "bn_seg1"),
    ("seg_conv2", 512, 256, "bn_seg2"),
    ("seg_conv3", 256, 128, "bn_seg3"),
    ("seg_conv4", 128, None, None),
]
BNS = [(bn, cout) for _, _, cout, bn in CONVS if bn]


def param_layout(num_classes: int, input_dim: int = 4):
    """[(name, shape)] of the parameters in registration order (== module.parameters())."""
    out = []
    for conv, cin, cout, _ in CONVS:
        cin = input_dim if cin is None else cin
        cout = num_classes if cout is None else cout
        out += [(f"{conv}.weight", (cout, cin, 1)), (f"{conv}.bias", (cout,))]
    for bn, c in BNS:
        out += [(f"{bn}.weight", (c,)), (f"{bn}.bias", (c,))]
    return out


# Flat fp32 buffers (parameters / gradients, optim.flatten_parameters): the parameters are
# grouped by when the backward finishes their gradients, so each all-reduce bucket (§8 e) is
# one contiguous range issued as soon as the backward has written it:
#   "seg"    seg_conv1..seg_conv4 + the EXTRA tail (loss numerator, CE weight sum, valid
#            count): ready once seg_conv1's local input/weight gradient has run;
#   "global" global_feat: ready after the Gram-form weight gradient (mid-backward);
#   "tail"   the 9 BatchNorms and conv1..conv5: ready at the end.
FLAT_EXTRA = 4
_SEG = ("seg_conv1", "seg_conv2", "seg_conv3", "seg_conv4")
_EARLY_CONVS = ("conv1", "conv2", "conv3", "conv4", "conv5")


def flat_layout(num_classes: int, input_dim: int = 4):
    """[(name, shape)] in flat-buffer order (see above); registration order is param_layout."""
    reg = dict(param_layout(num_classes, input_dim))
    names = [f"{bn}.{w}" for bn, _ in BNS for w in ("weight", "bias")]
    for conv in _EARLY_CONVS + ("global_feat",) + _SEG:
        names += [f"{conv}.weight", f"{conv}.bias"]
    return [(n, reg[n]) for n in names]


def flat_offsets(num_classes: int, input_dim: int = 4):
    """name -> element offset in the flat buffers; the EXTRA tail starts at the total."""
    offs, off = {}, 0
    for n, shape in flat_layout(num_classes, input_dim):
        offs[n] = off
        off += int(torch.Size(shape).numel())
    return offs, off


def bucket_ranges(num_classes: int, input_dim: int = 4):
    """Gradient all-reduce buckets: name -> [lo, hi) element range of the flat gradient
    buffer (which carries FLAT_EXTRA scalars after the parameters)."""
    offs, total = flat_offsets(num_classes, input_dim)
    return {"seg": (offs["seg_conv1.weight"], total + FLAT_EXTRA),
            "global": (offs["global_feat.weight"], offs["seg_conv1.weight"]),
            "tail": (0, offs["global_feat.weight"])}


def check_dims(num_classes: int, input_dim: int):
    """The reference accepts any input_dim / num_classes (P:66-83; num_classes comes from the
    data, P:153); the kernels cover input_dim 1..8 (conv1 is unrolled over K) and 1..256
    classes (the head keeps seg_conv4's fp32 weight in LDS: 128 KB at 256 classes)."""
    if not 1 <= int(input_dim) <= MAX_INPUT_DIM:
        raise ValueError(f"pcs_amd supports input_dim 1..{MAX_INPUT_DIM} (the reference's points carry "
                         f"4: x, y, z, e); got {input_dim}")
    if not 1 <= int(num_classes) <= MAX_CLASSES:
        raise ValueError(f"pcs_amd supports 1..{MAX_CLASSES} classes (seg_conv4 + CE head kernel); "
                         f"got {num_classes}")


def _dt(dtype: str):
    """(C-ABI dtype, torch dtype) of the stored activations.  "fp8" is the bf16 path with the
    wide layer (a5 = relu(bn5(y5)) and global_feat's operands) in fp8 e4m3."""
    if dtype == "fp32":
        return L.F32, torch.float32
    if dtype in ("bf16", "fp8"):
        return L.BF16, torch.bfloat16
    raise ValueError(f"compute dtype must be 'fp32', 'bf16' or 'fp8', got {dtype!r}")


@dataclass
class BNCoef:
    """Per-BN vectors produced by the forward finalisation (all fp32 [C] / [B,C])."""
    mean: torch.Tensor
    rstd: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor
    scene_sum: torch.Tensor


@dataclass
class Saved:
    """Everything the backward needs from one forward."""
    B: int
    N: int
    train: bool
    ys: dict = field(default_factory=dict)        # conv name -> Y tensor [M, C]
    bn: dict = field(default_factory=dict)        # bn name -> BNCoef
    masks: tuple = (None, None)                   # dropout keep bits (seg1 out, seg2 out)
    g: torch.Tensor = None
    am: torch.Tensor = None
    ysel: torch.Tensor = None
    x: torch.Tensor = None
    logits: torch.Tensor = None
    wc: dict = None                               # cast weights used by this pass
    gram4: tuple = None                           # (G, S) of a4 when the forward computed it
    gram2: object = None                          # conv3's per-chunk [G | S] records of a2 (fused seg12)
    a5_colsum: torch.Tensor = None                # bf16: per-chunk column sums of a5 (conv5 epilogue)
    mask_bufs: tuple = None                       # dropout keep bits drawn on the side stream
    gram5: tuple = None                           # bf16/fp8: (G, per-scene S, workspace) of a5, from the forward
    wg_eff: torch.Tensor = None                   # global_feat's weight as the forward GEMM saw it (fp32)
    sbias_s1: torch.Tensor = None                 # [B, 512] per-scene (centred) bias of the stored seg_conv1 output
    mask_ready: object = None                     # torch.cuda.Event recorded after them


class Engine:
    """Launches the PointNetSegmentation kernels for one compute dtype and device."""

    def __init__(self, num_classes: int, dtype: str = "fp32", input_dim: int = 4, eval_trunk: str = "fp32"):
        check_dims(num_classes, input_dim)
        if eval_trunk not in ("fp32", "bf16"):
            raise ValueError(f"eval_trunk must be 'fp32' or 'bf16', got {eval_trunk!r}")
        self.input_dim = input_dim
        self.C = num_classes
        self.dtype = dtype
        self.dt, self.tdt = _dt(dtype)
        # fp8: conv5 stores a5 as e4m3 and global_feat runs on MX-scaled fp8 MFMA (W rows
        # quantized with one E8M0 scale each, pcs_quant_fp8_rows), forward and input gradient
        self.fp8 = dtype == "fp8"
        self.a5_dt = L.FP8 if self.fp8 else self.dt
        # bf16 / fp8 EVAL forward: the narrow trunk conv1..conv4 (<= 128 channels, 10 % of the
        # activation bytes) stored and computed in fp32, conv5 on a 16-bit split of a4
        # (pcs_bnrelu_bf16); the trained network amplifies the trunk's bf16 rounding into
        # logit-margin error that moves mIoU by > 1e-3.  "bf16" keeps
        # the whole eval forward on bf16 storage (the training step's precision).
        self.eval_trunk = eval_trunk
        self.layout = param_layout(num_classes, input_dim)          # registration order
        self.numel = {n: int(torch.Size(s).numel()) for n, s in self.layout}
        self.offsets, self.total_params = flat_offsets(num_classes, input_dim)   # flat order
        self.buckets = bucket_ranges(num_classes, input_dim)
        self._geo = {}
        self._side = {}   # device -> side stream
        self.flags = 0       # L.FLAG_GENERIC forces the generic GEMM (cross-checks)
        self.timing = None   # dict tag -> [(start, end) torch.cuda.Event] when profiling
        self.timing_tags = None   # set of tags to bracket (None = every tagged launch)
        # test hooks for the global max-pool's rows (P:114): record_pool_rows keeps a copy of
        # the argmax rows [B, 1024] of the last forward in last_pool_rows; pool_rows_override
        # (int32 [B, 1024] global rows) replaces them before the backward routes the pooled
        # gradient, so a bf16 step can be compared with the fp32 step through the same rows
        # (tests/test_gpu_fullsize.py).  Never set on the product path.
        self.record_pool_rows = False
        self.last_pool_rows = None
        self.pool_rows_override = None
        # test hooks for the pre-pool backward at full size (tests/test_gpu_fullsize.py):
        # capture (a dict) receives the operands and outputs of global_feat's input gradient and
        # conv5's backward kernels; perturb = {"dz5": (c0, c1, scale)} scales columns c0..c1 of
        # dz5 after global_feat's input gradient (a simulated kernel error, the negative
        # control); {"a5": (rows, cols, value)} writes value into a5[rows, cols] after conv5's
        # forward (a diverged activation: NaN through the max-pool, tests/test_gpu_pool_nan.py).
        # Never set on the product path.
        self.capture = None
        self.perturb = None
        # bf16 / fp8 training forward: seg_conv1's local half and seg_conv2 in one streaming pass
        # (pcs_fwd_seg12, bn_seg1's statistics from the Gram of a2); False runs the two pcs_gemm
        # passes (cross-checks)
        self.fused_seg12 = True
        # bf16 training step: draw the dropout keep bits beside the Gram of a5 (bounded grid, in
        # its idle VALU issue) instead of at the start of the forward with a full grid
        self.draw_beside_gram = True
        # "paired" (default): pcs_dropout_bits (elements 2k, 2k + 1 share a byte pair of their
        # uniforms); "independent": pcs_dropout_bits_independent, i.i.d. keep bits as nn.Dropout
        # (P:96) at twice the Philox calls, drawn at the start of the forward (parity runs)
        self.dropout_draw = "paired"
        L.load()

    def _launch(self, tag, name, *args):
        """C-ABI call, bracketed by HIP events on the launch stream when timing is on."""
        if self.timing is None or tag is None or (self.timing_tags is not None and tag not in self.timing_tags):
            return L.call(name, *args)
        st = torch.cuda.Event(enable_timing=True)
        en = torch.cuda.Event(enable_timing=True)
        st.record()
        r = L.call(name, *args)
        en.record()
        self.timing.setdefault(tag, []).append((st, en))
        return r

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return L.stream_ptr()

    def _side_stream(self, dev):
        """A per-device HIP stream for work with no data dependence on the trunk (dropout bits)."""
        st = self._side.get(dev)
        if st is None:
            st = self._side.setdefault(dev, torch.cuda.Stream(device=dev))
        return st

    def geometry(self, B, N, K, ncols, pro=L.PRO_BNRELU, epi=L.EPI_FWD, dtype=None):
        """(chunks_per_scene, rows_per_chunk) of the kernel pcs_gemm picks for these args."""
        dtype = self.dt if dtype is None else dtype
        key = (B, N, K, ncols, pro, epi, self.flags, dtype)
        if key not in self._geo:
            a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=ncols, dtype=dtype,
                           prologue=pro, epilogue=epi, chunks_per_scene=0, flags=self.flags)
            rpc = L.load().pcs_gemm_geometry(ct.byref(a))
            if rpc <= 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            self._geo[key] = (a.chunks_per_scene, rpc)
        return self._geo[key]

    def _empty(self, *shape, dtype=None, device):
        return torch.empty(*shape, dtype=dtype or self.tdt, device=device)

    def cast_weights(self, P):
        """fp32 parameters -> compute-dtype W and W^T copies (every call: params may change)."""
        dev = P["conv2.weight"].device
        wc = {}
        s = self._stream()
        for conv, cin, cout, _ in CONVS:
            if conv in ("conv1", "seg_conv4"):
                continue
            W = P[f"{conv}.weight"]
            rows, ld = W.shape[0], W.shape[1]
            cols = 64 if conv == "seg_conv1" else ld     # seg_conv1: local half only
            Wc = self._empty(rows, cols, device=dev)
            WcT = self._empty(cols, rows, device=dev)
            L.call("pcs_cast_weight", L.ptr(W), rows, cols, ld, self.dt, L.ptr(Wc), L.ptr(WcT), s)
            wc[conv] = (Wc, WcT)
        if self.fp8:
            wc["global_feat_fp8"] = self._quant_fp8(P["global_feat.weight"])
        return wc

    def _quant_fp8(self, W):
        """(e4m3 rows, E8M0 row scales, fp32 dequantized copy) of an fp32 [rows, cols(, 1)]
        matrix."""
        W = W.reshape(W.shape[0], -1)
        rows, cols = W.shape
        dev = W.device
        Wq = torch.empty(rows, cols, dtype=torch.uint8, device=dev)
        sc = torch.empty(rows, dtype=torch.uint8, device=dev)
        deq = torch.empty(rows, cols, dtype=torch.float32, device=dev)
        L.call("pcs_quant_fp8_rows", L.ptr(W), rows, cols, W.stride(0), L.ptr(Wq), L.ptr(sc), L.ptr(deq),
               self._stream())
        return Wq, sc, deq

    def _bn_finalize(self, bnname, stats, B, N, C, cps, rpc, P, bufs, train, dev, offset=None):
        """BN coefficients for stored activations that omit ``offset`` (the conv bias)."""
        coef = BNCoef(*(torch.empty(C, dtype=torch.float32, device=dev) for _ in range(4)),
                      torch.empty(B, C, dtype=torch.float32, device=dev))
        g, b = P[f"{bnname}.weight"], P[f"{bnname}.bias"]
        if train:
            rm, rv = bufs.get(f"{bnname}.running_mean"), bufs.get(f"{bnname}.running_var")
            upd = int(rm is not None and rv is not None)
            L.call("pcs_bn_fwd_finalize", L.ptr(stats), B, N, C, cps, rpc, L.ptr(g), L.ptr(b),
                   L.ptr(offset), L.ptr(rm), L.ptr(rv), BN_MOMENTUM, BN_EPS, upd, L.ptr(coef.mean),
                   L.ptr(coef.rstd), L.ptr(coef.scale), L.ptr(coef.shift), L.ptr(coef.scene_sum),
                   self._stream())
        else:
            L.call("pcs_bn_eval_coefs", L.ptr(g), L.ptr(b), L.ptr(bufs[f"{bnname}.running_mean"]),
                   L.ptr(bufs[f"{bnname}.running_var"]), L.ptr(offset), BN_EPS, C, L.ptr(coef.scale),
                   L.ptr(coef.shift), self._stream())
        return coef

    def _gemm(self, B, N, K, ncols, pro, epi, A, W, C, **kw):
        tag = kw.pop("tag", None)
        dtype = kw.pop("dtype", self.dt)
        cps, _ = self.geometry(B, N, K, ncols, pro, epi, dtype)
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=K, Ncols=ncols, dtype=dtype,
                       prologue=pro, epilogue=epi, chunks_per_scene=cps,
                       flags=self.flags | kw.pop("extra_flags", 0),
                       A=L.ptr(A), W=L.ptr(W), C=L.ptr(C),
                       a_keep_scale=kw.pop("a_keep_scale", 1.0),
                       c_keep_scale=kw.pop("c_keep_scale", 1.0),
                       pool_ldw=kw.pop("pool_ldw", 0), pool_c=kw.pop("pool_c", 0), K1=kw.pop("K1", 0))
        for k, v in kw.items():
            setattr(a, k, L.ptr(v))
        self._launch(tag, "pcs_gemm", ct.byref(a), self._stream())

    def _wgrad(self, B, N, cout, cin, dy_mode, x_mode, dW, ldw=0, conv1=False, **kw):
        tag = kw.pop("tag", None)
        a = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=cout, Cin=cin, dtype=self.dt,
                        splits_per_scene=0, dy_mode=dy_mode, x_mode=x_mode,
                        x_keep_scale=kw.pop("x_keep_scale", 1.0), dW=L.ptr(dW), ldw=ldw,
                        flags=self.flags)
        for k, v in kw.items():
            setattr(a, k, L.ptr(v))
        fn = "pcs_conv1_wgrad" if conv1 else "pcs_wgrad"
        if conv1:
            a.splits_per_scene = max(1, min((1024 + B - 1) // B, (N + 255) // 256))
            nbytes = B * a.splits_per_scene * cout * cin * 4
        else:
            nbytes = L.load().pcs_wgrad_workspace(ct.byref(a))
        ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dW.device)
        a.partial = ws.data_ptr()
        self._launch(tag, fn, ct.byref(a), self._stream())
        return ws  # keep alive until the stream consumes it (caching allocator is stream-ordered)

    def _raw_gram(self):
        """bf16 / fp8 wide-layer path: a5 is stored post-ReLU, so global_feat's Gram reads it
        raw on the LDS-DMA kernel (pcs_gram_raw) with column sums from conv5's epilogue."""
        return self.dt == L.BF16 and not (self.flags & L.FLAG_GENERIC)

    def _rounded(self, W):
        """fp32 copy of W as the forward's compute-dtype GEMM saw it (pcs_round_weight)."""
        if self.dt == L.F32:
            return W
        out = torch.empty_like(W)
        L.call("pcs_round_weight", L.ptr(W), W.numel(), self.dt, L.ptr(out), self._stream())
        return out

    def _gram(self, Y, s_, t_, B, N, C, tag=None):
        """(G, S) = (a^T a, column sums of a) for a = relu(Y*s + t) (pcs_gram)."""
        dev = Y.device
        G = torch.empty(C, C, dtype=torch.float32, device=dev)
        S = torch.empty(C, dtype=torch.float32, device=dev)
        sps = ct.c_int32(0)
        nbytes = L.load().pcs_gram_workspace(B, N, C, self.dt, ct.byref(sps))
        ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dev)
        self._launch(tag, "pcs_gram", L.ptr(Y), L.ptr(s_), L.ptr(t_), B, N, C, self.dt, sps.value, L.ptr(ws),
                     L.ptr(G), L.ptr(S), self._stream())
        return G, S, ws

    # ------------------------------------------------------------------ forward
    def forward(self, P, bufs, x, *, train, masks=None, seed=0, head_mode=L.HEAD_FWD,
                labels=None, class_weight=None, wsum=None, want_logits=True, saved=None):
        """Forward pass.  P: name -> fp32 parameter tensor; bufs: BN running buffers.

        ``masks`` = (bits1 [M,64] u8, bits2 [M,32] u8) replays dropout keep bits; otherwise
        train mode draws them with Philox from ``seed``.  With ``head_mode=HEAD_CE`` the
        head kernel also computes the weighted CE loss and starts the backward (fused
        train step); returns the Saved context (plus head outputs in ``saved.head``).
        """
        if not x.is_cuda:
            raise RuntimeError("pcs_amd runs on a HIP device only (no CPU fallback)")
        dev = x.device
        B, N, D = x.shape
        if D != self.input_dim:
            raise ValueError(f"expected x of shape (B, N, {self.input_dim}), got {tuple(x.shape)}")
        M = B * N
        s = self._stream()
        x = x.contiguous().float()
        sv = Saved(B=B, N=N, train=train) if saved is None else saved
        sv.B, sv.N, sv.train, sv.x = B, N, train, x
        sv.gram4 = None   # (a reused Saved must not carry the previous pass's Gram)
        def draw_masks(max_wg=0):
            # Philox keep bits (ALU-bound, no data dependence) drawn on a side stream beside the
            # trunk's kernels; the stream waits for everything enqueued before (the buffers may
            # reuse memory the previous kernels still read) and seg_conv2 waits for it
            m1 = torch.empty(M, 64, dtype=torch.uint8, device=dev)
            m2 = torch.empty(M, 32, dtype=torch.uint8, device=dev)
            side = self._side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                ss = L.stream_ptr()
                if self.dropout_draw == "independent":
                    L.call("pcs_dropout_bits_independent", seed, 0, M, 512, DROPOUT_P, L.ptr(m1), ss)
                    L.call("pcs_dropout_bits_independent", seed, 1, M, 256, DROPOUT_P, L.ptr(m2), ss)
                else:
                    L.call("pcs_dropout_bits_bounded", seed, 0, M, 512, DROPOUT_P, L.ptr(m1), max_wg, ss)
                    L.call("pcs_dropout_bits_bounded", seed, 1, M, 256, DROPOUT_P, L.ptr(m2), max_wg, ss)
                sv.mask_ready = torch.cuda.Event()
                sv.mask_ready.record(side)
            m1.record_stream(side)
            m2.record_stream(side)
            sv.mask_bufs = (m1, m2)
        # bf16 / fp8 (stored-a5 Gram): draw beside the Gram of a5, MFMA-bound at 214 / 216 VGPRs x 2 waves per
        # SIMD, with three 256-thread workgroups per CU (24 VGPRs a wave: they fit beside it and
        # use its idle VALU issue; 0.77 ms per call against 0.83 with two, the Gram and the step
        # unchanged, tools/draw_wg.py); otherwise at the start of the forward with a full grid
        draw_beside_gram = (train and masks is None and self._raw_gram() and self.draw_beside_gram
                            and self.dropout_draw != "independent")
        if train and masks is None and not draw_beside_gram:
            draw_masks()
        sv.wc = wc = self.cast_weights(P)
        T = self.tdt

        def stats_buf(K, ncols):
            cps, rpc = self.geometry(B, N, K, ncols)
            return torch.empty(B * cps, ncols, 2, dtype=torch.float32, device=dev), cps, rpc

        def bnrelu(prev):
            c = sv.bn[prev]
            return dict(pa=c.scale, pb=c.shift)

        # Stored pre-BN activations omit the conv bias (BN cancels it exactly; it only
        # shifts running_mean), which keeps them centred: full precision in fp32/bf16.
        # bf16 / fp8 eval: conv1..conv4 in fp32 (self.eval_trunk, see __init__)
        trunk32 = not train and self.dt == L.BF16 and self.eval_trunk == "fp32"
        tdt = L.F32 if trunk32 else self.dt
        # conv1 (K=4)
        y1 = self._empty(M, 64, device=dev, dtype=torch.float32 if trunk32 else None)
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=D, Ncols=64, dtype=L.F32, chunks_per_scene=0,
                       flags=L.FLAG_GENERIC)
        rpc = L.load().pcs_gemm_geometry(ct.byref(a))    # conv1: generic 128-row geometry
        cps = a.chunks_per_scene
        st = torch.empty(B * cps, 64, 2, dtype=torch.float32, device=dev) if train else None
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=D, Ncols=64, dtype=tdt,
                       chunks_per_scene=cps, A=L.ptr(x), W=L.ptr(P["conv1.weight"]),
                       C=L.ptr(y1), bias=None, stats=L.ptr(st))
        self._launch("fwd:conv1", "pcs_conv1_fwd", ct.byref(a), s)
        sv.ys["conv1"] = y1
        sv.bn["bn1"] = self._bn_finalize("bn1", st, B, N, 64, cps, rpc, P, bufs, train, dev,
                                         offset=P["conv1.bias"])

        def layer(conv, src_conv, src_bn, K, ncols, bnname, offset, **kw):
            st, cps, rpc = stats_buf(K, ncols) if train else (None, 0, 0)
            if kw.get("dtype") == L.F32:       # the eval path's fp32 trunk
                y = self._empty(M, ncols, device=dev, dtype=torch.float32)
                self._gemm(B, N, K, ncols, L.PRO_BNRELU, L.EPI_FWD, sv.ys[src_conv], P[f"{conv}.weight"], y,
                           stats=st, tag=f"fwd:{conv}", **bnrelu(src_bn), **kw)
            elif "A_raw" in kw:                # bf16 GEMM on an activation bridged from the trunk
                y = self._empty(M, ncols, device=dev)
                self._gemm(B, N, K, ncols, L.PRO_RAW, L.EPI_FWD, kw.pop("A_raw"), wc[conv][0], y,
                           stats=st, tag=f"fwd:{conv}", **kw)
            else:
                y = self._empty(M, ncols, device=dev)
                self._gemm(B, N, K, ncols, L.PRO_BNRELU, L.EPI_FWD, sv.ys[src_conv], wc[conv][0], y,
                           stats=st, tag=f"fwd:{conv}", **bnrelu(src_bn), **kw)
            sv.ys[conv] = y
            sv.bn[bnname] = self._bn_finalize(bnname, st, B, N, ncols, cps, rpc, P, bufs, train,
                                              dev, offset=offset)
            return y

        tkw = {"dtype": L.F32} if trunk32 else {}
        layer("conv2", "conv1", "bn1", 64, 64, "bn2", P["conv2.bias"], **tkw)
        # the fused seg_conv1 + seg_conv2 forward takes bn_seg1's statistics from the Gram of a2,
        # which conv3's streaming pass forms from the operand it already has in LDS
        fused12 = train and self.dt == L.BF16 and not (self.flags & L.FLAG_GENERIC) and self.fused_seg12
        gkw = {}
        if fused12:
            cps3, _ = self.geometry(B, N, 64, 64)
            sv.gram2 = torch.empty(B * cps3, 64 * 64 + 64, dtype=torch.float32, device=dev)
            gkw = {"gram": sv.gram2}
        layer("conv3", "conv2", "bn2", 64, 64, "bn3", P["conv3.bias"], **tkw, **gkw)
        layer("conv4", "conv3", "bn3", 64, 128, "bn4", P["conv4.bias"], **tkw)

        def bridge(conv, bn, K, split):
            """relu(bn(Y)) of an fp32 trunk output as bf16 (split: [hi | lo], pcs_bnrelu_bf16)."""
            out = self._empty(M, 2 * K if split else K, device=dev)
            c = sv.bn[bn]
            L.call("pcs_bnrelu_bf16", L.ptr(sv.ys[conv]), M, K, L.ptr(c.scale), L.ptr(c.shift), int(split),
                   L.ptr(out), s)
            return out

        # conv5 (P:110): bn5's statistics first, then the GEMM with bn5 + ReLU applied in the
        # epilogue, storing a5 = relu(bn5(y5)) for global_feat.  fp32: a statistics-only pass
        # of the GEMM.  bf16: from the Gram of a4 (which conv5's weight gradient needs anyway),
        # mean = W5 S4 / M and M2 = w (G4 - S4 S4^T / M) w^T per channel.
        st, cps, rpc = (None, 0, 0)
        if train and self.dt == L.BF16:
            c4 = sv.bn["bn4"]
            sv.gram4 = self._gram(sv.ys["conv4"], c4.scale, c4.shift, B, N, 128, tag="fwd_stats:conv5")
            st, cps, rpc = torch.empty(B, 1024, 2, dtype=torch.float32, device=dev), 1, N
            L.call("pcs_bn_stats_from_gram", L.ptr(sv.gram4[0]), L.ptr(sv.gram4[1]), M, L.ptr(wc["conv5"][0]),
                   self.dt, 128, 1024, 128, B, L.ptr(st), s)
        elif train:
            st, cps, rpc = stats_buf(128, 1024)
            self._gemm(B, N, 128, 1024, L.PRO_BNRELU, L.EPI_FWD, sv.ys["conv4"], wc["conv5"][0], None,
                       stats=st, tag="fwd_stats:conv5", **bnrelu("bn4"))
        sv.bn["bn5"] = self._bn_finalize("bn5", st, B, N, 1024, cps, rpc, P, bufs, train, dev,
                                         offset=P["conv5.bias"])
        a5 = self._empty(M, 1024, device=dev, dtype=torch.uint8 if self.fp8 else None)
        c5 = sv.bn["bn5"]
        # bf16: the epilogue also sums a5's columns per chunk (S of global_feat's Gram-form
        # weight gradient; the LDS-DMA Gram kernel computes G only)
        sv.a5_colsum = None
        if train and self._raw_gram():
            cps5c, _ = self.geometry(B, N, 128, 1024, L.PRO_BNRELU, L.EPI_BNRELU)
            sv.a5_colsum = torch.empty(B * cps5c, 1024, 2, dtype=torch.float32, device=dev)
        if trunk32:
            # a4 to 16 significant bits: [hi | lo] (K = 256) against [W5 | W5]
            W5s = torch.cat([wc["conv5"][0], wc["conv5"][0]], dim=1)
            self._gemm(B, N, 256, 1024, L.PRO_RAW, L.EPI_BNRELU, bridge("conv4", "bn4", 128, True), W5s, a5,
                       es=c5.scale, et=c5.shift, tag="fwd:conv5", extra_flags=L.FLAG_C_FP8 if self.fp8 else 0)
        else:
            self._gemm(B, N, 128, 1024, L.PRO_BNRELU, L.EPI_BNRELU, sv.ys["conv4"], wc["conv5"][0], a5,
                       es=c5.scale, et=c5.shift, stats=sv.a5_colsum, tag="fwd:conv5",
                       extra_flags=L.FLAG_C_FP8 if self.fp8 else 0, **bnrelu("bn4"))
        if self.perturb is not None and "a5" in self.perturb:
            rows, cols, value = self.perturb["a5"]
            if self.fp8:   # e4m3 bytes: 0x7f is its NaN
                a5[rows, cols] = 0x7f if value != value else int(torch.tensor(value).to(torch.float8_e4m3fn).view(torch.uint8))
            else:
                a5[rows, cols] = value
        sv.ys["a5"] = a5

        # global_feat (P:113-114): a5 W^T with max-pool partials (and, on the fp32 / generic
        # paths, BN statistics) in the epilogue; the 1024-wide output itself is never stored.
        # bf16 / fp8: bn_global's statistics come from the Gram of a5 -- computed here rather
        # than in the backward, whose Gram-form weight gradient reuses it -- and conv5's
        # per-chunk column sums (pcs_bn_stats_from_gram_scenes), so the LDS-DMA forward runs
        # the max-pool epilogue only.
        cps_g, rpc_g = self.geometry(B, N, 1024, 1024, L.PRO_RAW, L.EPI_FWD)
        pool = torch.empty(B * cps_g, 1024, 4, dtype=torch.float32, device=dev)
        sv.gram5 = None
        if train and self._raw_gram():
            Wg = P["global_feat.weight"]
            sv.wg_eff = wc["global_feat_fp8"][2] if self.fp8 else self._rounded(Wg.reshape(1024, -1))
            G5 = torch.empty(1024, 1024, dtype=torch.float32, device=dev)
            nbytes = L.load().pcs_gram_raw_workspace(M, 1024)
            if nbytes < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            gws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            if draw_beside_gram:
                draw_masks(3 * torch.cuda.get_device_properties(dev).multi_processor_count)
            self._launch("wgrad:global_feat", "pcs_gram_raw", L.ptr(a5), M, 1024, self.a5_dt, L.ptr(gws), nbytes,
                         L.ptr(G5), s)
            # per-scene column sums of a5 from conv5's per-chunk partials (chunks are scene-aligned)
            Sb2 = torch.empty(B, 1024, 2, dtype=torch.float32, device=dev)
            L.call("pcs_reduce_partials_grouped", L.ptr(sv.a5_colsum), B, cps5c, 2048, 1.0, L.ptr(Sb2), s)
            Sb = Sb2[..., 0].contiguous()
            st = torch.empty(B, 1024, 2, dtype=torch.float32, device=dev)
            qbytes = L.load().pcs_bn_stats_from_gram_scenes_workspace(1024, 1024)
            qws = torch.empty(qbytes // 8, dtype=torch.float64, device=dev)
            self._launch("stats:global_feat", "pcs_bn_stats_from_gram_scenes", L.ptr(G5), L.ptr(Sb), N, L.ptr(sv.wg_eff), L.F32, 1024, 1024,
                         1024, B, L.ptr(qws), qbytes, L.ptr(st), s)
            sv.gram5 = (G5, Sb, gws)
            st_g, cps_st, rpc_st = None, 1, N
        else:
            st = torch.empty(B * cps_g, 1024, 2, dtype=torch.float32, device=dev) if train else None
            st_g, cps_st, rpc_st = st, cps_g, rpc_g
        # (es = bn_global's gamma: its sign tells the pool which extremum pcs_pool_finalize uses;
        # without statistics on the LDS-DMA kernel, W's rows come pre-multiplied by that sign,
        # PCS_FLAG_POOL_SIGNED_W, and the pool keeps a plain column max)
        gamma_g = P["bn_global.weight"]
        Wf = wc["global_feat_fp8"][0] if self.fp8 else wc["global_feat"][0]
        sflag = 0
        if st_g is None and self._raw_gram() and not (self.flags & L.FLAG_NO_GLDS):
            Wsg = torch.empty_like(Wf)
            L.call("pcs_sign_rows", L.ptr(Wf), L.FP8 if self.fp8 else self.dt, 1024, 1024, L.ptr(gamma_g),
                   L.ptr(Wsg), s)
            Wf, sflag = Wsg, L.FLAG_POOL_SIGNED_W
        if self.fp8:
            self._gemm(B, N, 1024, 1024, L.PRO_RAW, L.EPI_FWD, a5, Wf, None, stats=st_g, pool=pool, es=gamma_g,
                       w_scale=wc["global_feat_fp8"][1], extra_flags=L.FLAG_AW_FP8 | sflag, tag="fwd:global_feat")
        else:
            self._gemm(B, N, 1024, 1024, L.PRO_RAW, L.EPI_FWD, a5, Wf, None, stats=st_g, pool=pool, es=gamma_g,
                       extra_flags=sflag, tag="fwd:global_feat")
        sv.bn["bn_global"] = self._bn_finalize("bn_global", st, B, N, 1024, cps_st, rpc_st, P, bufs,
                                               train, dev, offset=P["global_feat.bias"])
        cg = sv.bn["bn_global"]
        sv.g = torch.empty(B, 1024, dtype=torch.float32, device=dev)
        sv.am = torch.empty(B, 1024, dtype=torch.int32, device=dev)
        sv.ysel = torch.empty(B, 1024, dtype=torch.float32, device=dev)
        L.call("pcs_pool_finalize", L.ptr(pool), B, N, 1024, cps_g, L.ptr(cg.scale), L.ptr(cg.shift),
               L.ptr(sv.g), L.ptr(sv.am), L.ptr(sv.ysel), s)
        if self.record_pool_rows:
            self.last_pool_rows = sv.am.clone()
        if self.pool_rows_override is not None:
            sv.am.copy_(self.pool_rows_override)

        # seg_conv1 = local 64->512 GEMM + per-scene bias (W_global . g_b + b)   P:117-123
        # the per-scene bias is centred over the scenes; its mean joins the BN offset
        sbias = torch.empty(B, 512, dtype=torch.float32, device=dev)
        soff = torch.empty(512, dtype=torch.float32, device=dev)
        Ws1 = P["seg_conv1.weight"]
        L.call("pcs_scene_gemv", L.ptr(sv.g), B, 1024, L.ptr(Ws1), Ws1.shape[1], 64,
               L.ptr(P["seg_conv1.bias"]), 512, L.ptr(sbias), L.ptr(soff), s)
        sv.sbias_s1 = sbias   # the stored Y'_seg1 = a2 W_l^T + sbias[b] (the folded backward)
        if fused12:
            pass   # with seg_conv2 below (pcs_fwd_seg12)
        elif trunk32:
            layer("seg_conv1", "conv2", "bn2", 64, 512, "bn_seg1", soff, scene_bias=sbias,
                  A_raw=bridge("conv2", "bn2", 64, False))
        else:
            layer("seg_conv1", "conv2", "bn2", 64, 512, "bn_seg1", soff, scene_bias=sbias)

        # dropout keep bits (P:124, P:126)
        if train:
            if masks is not None:
                m1, m2 = masks
                # the kernels read M x 512 / M x 256 keep bits: a mask for another batch
                # shape (e.g. a DataParallel replica's chunk) would be read out of bounds
                if (tuple(m1.shape) != (M, 64) or tuple(m2.shape) != (M, 32) or m1.dtype != torch.uint8
                        or m2.dtype != torch.uint8 or m1.device != dev or m2.device != dev):
                    raise ValueError(f"dropout masks must be uint8 [{M}, 64] and [{M}, 32] on {dev}, got "
                                     f"{tuple(m1.shape)} {m1.dtype} and {tuple(m2.shape)} {m2.dtype}")
                m1, m2 = m1.contiguous(), m2.contiguous()
            else:
                m1, m2 = sv.mask_bufs
                torch.cuda.current_stream(dev).wait_event(sv.mask_ready)   # drawn on the side stream
            sv.masks = (m1, m2)
            keep = 1.0 / (1.0 - DROPOUT_P)
        else:
            m1 = m2 = None
            sv.masks = (None, None)
            keep = 1.0
        if fused12:
            self._seg12(P, bufs, sv, wc, sbias, soff, m1, keep)
        else:
            layer("seg_conv2", "seg_conv1", "bn_seg1", 512, 256, "bn_seg2", P["seg_conv2.bias"],
                  a_mask=m1, a_keep_scale=keep)
        layer("seg_conv3", "seg_conv2", "bn_seg2", 256, 128, "bn_seg3", P["seg_conv3.bias"],
              a_mask=m2, a_keep_scale=keep)

        # head: seg_conv4 (+ CE and the start of the backward when fused)
        sv.logits = (torch.empty(B, N, self.C, dtype=torch.float32, device=dev)
                     if want_logits else None)
        if head_mode == L.HEAD_CE:
            sv.head = self._head(P, sv, L.HEAD_CE, labels=labels, class_weight=class_weight,
                                 wsum=wsum)
        else:
            self._head(P, sv, L.HEAD_FWD)
        return sv

    def _seg12(self, P, bufs, sv, wc, sbias, soff, m1, keep):
        """seg_conv1 (local half + scene bias) and seg_conv2 forward in one pass (P:117-125;
        pcs_fwd_seg12).  bn_seg1's batch statistics come first, from the Gram of a2 =
        relu(bn2(y2)) and its per-scene column sums (pcs_gram, pcs_bn_stats_gram_sbias), with
        the bf16-rounded W_l the pass multiplies by."""
        B, N = sv.B, sv.N
        M = B * N
        dev = sv.x.device
        s = self._stream()
        c2 = sv.bn["bn2"]
        # conv3's per-chunk [G | S] records of a2 -> per scene, then G2 over the scenes
        rec = 64 * 64 + 64
        cps3 = sv.gram2.shape[0] // B
        per_scene = torch.empty(B, rec, dtype=torch.float32, device=dev)
        L.call("pcs_reduce_partials_grouped", L.ptr(sv.gram2), B, cps3, rec, 1.0, L.ptr(per_scene), s)
        tot = torch.empty(rec, dtype=torch.float32, device=dev)
        L.call("pcs_reduce_partials", L.ptr(per_scene), B, rec, 1.0, L.ptr(tot), 1, rec, s)
        G2 = tot[:64 * 64]
        Sb = per_scene[:, 64 * 64:].contiguous()
        Ws1 = P["seg_conv1.weight"]
        Ws1_r = self._rounded(Ws1)
        st1 = torch.empty(B, 512, 2, dtype=torch.float32, device=dev)
        L.call("pcs_bn_stats_gram_sbias", L.ptr(G2), L.ptr(Sb), B, N, L.ptr(Ws1_r), Ws1.shape[1], 64, 512,
               L.ptr(sbias), L.ptr(st1), s)
        sv.bn["bn_seg1"] = c1 = self._bn_finalize("bn_seg1", st1, B, N, 512, 1, N, P, bufs, True, dev, offset=soff)
        y1 = self._empty(M, 512, device=dev)
        y2 = self._empty(M, 256, device=dev)
        a = L.Seg12Args(num_scenes=B, scene_rows=N, chunks_per_scene=0, y2=L.ptr(sv.ys["conv2"]), s2=L.ptr(c2.scale),
                        t2=L.ptr(c2.shift), W1=L.ptr(wc["seg_conv1"][0]), sbias=L.ptr(sbias), Y1=L.ptr(y1),
                        s1=L.ptr(c1.scale), t1=L.ptr(c1.shift), keep1=L.ptr(m1), keep_scale=keep,
                        W2=L.ptr(wc["seg_conv2"][0]), Y2=L.ptr(y2))
        rpc = L.load().pcs_fwd_seg12_geometry(ct.byref(a))
        if rpc <= 0:
            raise L.PcsError(L.load().pcs_last_error().decode())
        cps = a.chunks_per_scene
        st2 = torch.empty(B * cps, 256, 2, dtype=torch.float32, device=dev)
        a.stats = L.ptr(st2)
        self._launch("fwd:seg_conv1+2", "pcs_fwd_seg12", ct.byref(a), s)
        sv.ys["seg_conv1"], sv.ys["seg_conv2"] = y1, y2
        sv.bn["bn_seg2"] = self._bn_finalize("bn_seg2", st2, B, N, 256, cps, rpc, P, bufs, True, dev,
                                             offset=P["seg_conv2.bias"])

    def _head(self, P, sv, mode, labels=None, class_weight=None, wsum=None, dlogits=None):
        """seg_conv4 + (CE | given dlogits) + head backward; returns the backward buffers."""
        B, N = sv.B, sv.N
        dev = sv.x.device
        c3 = sv.bn["bn_seg3"]
        ha = L.HeadArgs(num_scenes=B, scene_rows=N, Cin=128, num_classes=self.C, dtype=self.dt,
                        mode=mode, chunks_per_scene=0, Y=L.ptr(sv.ys["seg_conv3"]),
                        s=L.ptr(c3.scale), t=L.ptr(c3.shift), W=L.ptr(P["seg_conv4.weight"]),
                        bias=L.ptr(P["seg_conv4.bias"]),
                        logits=L.ptr(sv.logits) if mode != L.HEAD_BWD else None)
        hb = None
        if mode != L.HEAD_FWD:
            L.load().pcs_head_geometry(ct.byref(ha))
            nch = B * ha.chunks_per_scene
            hb = dict(dZ=torch.empty(B * N * 1024, dtype=self.tdt, device=dev),
                      stats=torch.empty(nch, 128, 2, dtype=torch.float32, device=dev),
                      wpartial=torch.empty(nch, self.C * 129, dtype=torch.float32, device=dev),
                      loss_partial=torch.empty(nch, dtype=torch.float32, device=dev),
                      cps=ha.chunks_per_scene, nch=nch)
            ha.dZ, ha.stats = L.ptr(hb["dZ"]), L.ptr(hb["stats"])
            ha.wpartial, ha.loss_partial = L.ptr(hb["wpartial"]), L.ptr(hb["loss_partial"])
            ha.mean, ha.rstd = L.ptr(c3.mean), L.ptr(c3.rstd)
        if mode == L.HEAD_CE:
            ha.labels, ha.class_weight, ha.wsum = L.ptr(labels), L.ptr(class_weight), L.ptr(wsum)
        if mode == L.HEAD_BWD:
            dl = dlogits.reshape(B * N, self.C) if dlogits.dim() == 3 else dlogits
            if dl.dtype != torch.float32:
                dl = dl.float()
            ha.dlogits = L.ptr(dl)
            ha.dl_stride_row, ha.dl_stride_col = dl.stride(0), dl.stride(1)
            hb["dl"] = dl
        self._launch(f"head:{mode}", "pcs_head", ct.byref(ha), self._stream())
        return hb

    # ------------------------------------------------------------------ backward
    def backward(self, P, sv, gflat, dlogits=None, on_bucket=None):
        """Backward pass: every parameter gradient is written into the flat fp32 buffer
        ``gflat`` (flat order, see flat_layout).  Uses the head buffers of a fused CE
        forward, or runs the head backward on caller-supplied ``dlogits``.  ``on_bucket(name)``
        is called as soon as the kernels writing gradient bucket ``name`` (bucket_ranges)
        have been enqueued, so a data-parallel caller can start its all-reduce there."""
        bucket = on_bucket or (lambda name: None)
        if not sv.train:
            raise RuntimeError("backward needs a train-mode forward (BatchNorm batch statistics)")
        B, N = sv.B, sv.N
        M = B * N
        dev = sv.x.device
        s = self._stream()
        wc = sv.wc
        G = lambda name: gflat[self.offsets[name]:]   # noqa: E731  (pointer at a param's slot)
        hb = self._head(P, sv, L.HEAD_BWD, dlogits=dlogits) if dlogits is not None else sv.head
        keep = 1.0 / (1.0 - DROPOUT_P)
        m1, m2 = sv.masks

        # seg_conv4: weight and bias are adjacent in the flat buffer
        L.call("pcs_reduce_partials", L.ptr(hb["wpartial"]), hb["nch"], self.C * 129, 1.0,
               L.ptr(G("seg_conv4.weight")), self.C * 129, self.C * 129, s)

        coefs = {}

        def bn_bwd(bnname, conv, stats, cps, scene_s1=None):
            fc = sv.bn[bnname]
            C = fc.mean.shape[0]
            al, be, ga = (torch.empty(C, dtype=torch.float32, device=dev) for _ in range(3))
            L.call("pcs_bn_bwd_finalize", L.ptr(stats), B, N, C, cps, L.ptr(fc.mean), L.ptr(fc.rstd),
                   L.ptr(P[f"{bnname}.weight"]), L.ptr(fc.scene_sum), L.ptr(al), L.ptr(be), L.ptr(ga),
                   L.ptr(G(f"{bnname}.weight")), L.ptr(G(f"{bnname}.bias")),
                   L.ptr(G(f"{conv}.bias")), L.ptr(scene_s1), s)
            coefs[bnname] = (al, be, ga)

        bn_bwd("bn_seg3", "seg_conv3", hb["stats"], hb["cps"])

        bufA = hb["dZ"]
        bufB = torch.empty(M * 1024, dtype=self.tdt, device=dev)
        keepalive = []

        def dgrad(conv, bn, cin, cout, dz, ycur, prev_conv, prev_bn, out, c_mask=None,
                  addend=None):
            al, be, ga = coefs[bn]
            pc = sv.bn[prev_bn]
            cps, _ = self.geometry(B, N, cout, cin, L.PRO_BWD, L.EPI_DGRAD)
            st = torch.empty(B * cps, cin, 2, dtype=torch.float32, device=dev)
            self._gemm(B, N, cout, cin, L.PRO_BWD, L.EPI_DGRAD, dz, wc[conv][1], out,
                       A2=ycur, pa=al, pb=be, pc=ga, Yp=sv.ys[prev_conv], es=pc.scale, et=pc.shift,
                       emean=pc.mean, erstd=pc.rstd, c_mask=c_mask,
                       c_keep_scale=keep if c_mask is not None else 1.0, addend=addend, stats=st,
                       tag=f"dgrad:{conv}")
            return st, cps

        def wgrad(conv, bn, cin, cout, dz, ycur, prev_conv, prev_bn, x_mask=None, ldw=0):
            al, be, ga = coefs[bn]
            pc = sv.bn[prev_bn]
            keepalive.append(self._wgrad(
                B, N, cout, cin, L.PRO_BWD, L.PRO_BNRELU, G(f"{conv}.weight"), ldw=ldw, tag=f"wgrad:{conv}", dZ=dz,
                Y=ycur, alpha=al, beta=be, gamma=ga, X=sv.ys[prev_conv], s=pc.scale, t=pc.shift,
                x_mask=x_mask, x_keep_scale=keep if x_mask is not None else 1.0))

        def dgrad_wgrad(conv, bn, cin, cout, dz, ycur, prev_conv, prev_bn, out, c_mask=None,
                        addend=None):
            """Both gradients of one layer in one pass (csrc/fused_bwd.hip) where the fused
            kernel covers the shape (bf16); otherwise the pcs_gemm(DGRAD) + pcs_wgrad pair."""
            if self.dt == L.BF16 and not (self.flags & L.FLAG_GENERIC):
                al, be, ga = coefs[bn]
                pc = sv.bn[prev_bn]
                a = L.GemmArgs(num_scenes=B, scene_rows=N, K=cout, Ncols=cin, dtype=self.dt,
                               prologue=L.PRO_BWD, epilogue=L.EPI_DGRAD, chunks_per_scene=0,
                               flags=self.flags, A=L.ptr(dz), W=L.ptr(wc[conv][1]), C=L.ptr(out),
                               a_keep_scale=1.0, c_keep_scale=keep if c_mask is not None else 1.0)
                for k, v in dict(A2=ycur, pa=al, pb=be, pc=ga, Yp=sv.ys[prev_conv], es=pc.scale,
                                 et=pc.shift, emean=pc.mean, erstd=pc.rstd, c_mask=c_mask,
                                 addend=addend).items():
                    setattr(a, k, L.ptr(v))
                nbytes = L.load().pcs_dgrad_wgrad_bn_workspace(ct.byref(a))
                if nbytes > 0:
                    cps = a.chunks_per_scene
                    st = torch.empty(B * cps, cin, 2, dtype=torch.float32, device=dev)
                    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
                    a.stats = L.ptr(st)
                    self._launch(f"dgrad+wgrad:{conv}", "pcs_dgrad_wgrad_bn", ct.byref(a), L.ptr(ws),
                                 L.ptr(G(f"{conv}.weight")), 0, s)
                    keepalive.append(ws)
                    return st, cps
            st, cps = dgrad(conv, bn, cin, cout, dz, ycur, prev_conv, prev_bn, out, c_mask=c_mask,
                            addend=addend)
            wgrad(conv, bn, cin, cout, dz, ycur, prev_conv, prev_bn, x_mask=c_mask)
            return st, cps

        ys = sv.ys
        # seg_conv3 (input: dropout(relu(bn_seg2(y_s2))))
        dz_s3 = bufA
        st, cps = dgrad_wgrad("seg_conv3", "bn_seg3", 256, 128, dz_s3, ys["seg_conv3"], "seg_conv2",
                              "bn_seg2", bufB, c_mask=m2)
        bn_bwd("bn_seg2", "seg_conv2", st, cps)
        # seg_conv2 (input: dropout(relu(bn_seg1(y_s1))))
        dz_s2 = bufB
        st, cps = dgrad_wgrad("seg_conv2", "bn_seg2", 512, 256, dz_s2, ys["seg_conv2"], "seg_conv1",
                              "bn_seg1", bufA, c_mask=m1)
        scene_s1 = torch.empty(B, 512, dtype=torch.float32, device=dev)
        bn_bwd("bn_seg1", "seg_conv1", st, cps, scene_s1=scene_s1)
        dz_s1 = bufA

        # repeat/cat + max-pool + bn_global backward (P:113-120)
        a1, b1, g1 = coefs["bn_seg1"]
        cg = sv.bn["bn_global"]
        ag, bg, gg = (torch.empty(1024, dtype=torch.float32, device=dev) for _ in range(3))
        sp = torch.empty(B, 1024, dtype=torch.float32, device=dev)
        csum = torch.empty(B, 512, dtype=torch.float32, device=dev)
        Ws1 = P["seg_conv1.weight"]
        pa = L.PoolBwdArgs(
            num_scenes=B, scene_rows=N, Cs=512, Cg=1024, col_off=64,
            s1_alpha=L.ptr(a1), s1_beta=L.ptr(b1), s1_gamma=L.ptr(g1), s1_scene_s1=L.ptr(scene_s1),
            s1_scene_sum=L.ptr(sv.bn["bn_seg1"].scene_sum), W_s1=L.ptr(Ws1), ldw=Ws1.shape[1],
            g=L.ptr(sv.g), ysel=L.ptr(sv.ysel), g_mean=L.ptr(cg.mean), g_rstd=L.ptr(cg.rstd),
            g_gamma=L.ptr(P["bn_global.weight"]), g_scene_sum=L.ptr(cg.scene_sum),
            dW_s1_global=L.ptr(G("seg_conv1.weight")), csum=L.ptr(csum), alpha=L.ptr(ag),
            beta_c=L.ptr(bg), gamma_c=L.ptr(gg), dgamma=L.ptr(G("bn_global.weight")),
            dbeta=L.ptr(G("bn_global.bias")), dbias=L.ptr(G("global_feat.bias")), sp=L.ptr(sp))
        L.call("pcs_pool_bwd", ct.byref(pa), s)

        # seg_conv1 local half: dA2 contribution (raw) and dW[:, :64]
        dA2 = torch.empty(M, 64, dtype=self.tdt, device=dev)
        if self.dt == L.BF16 and not (self.flags & L.FLAG_GENERIC):
            # folded form, one pass over dz_s1 and y2 (csrc/fused_bwd.hip): with dy = a1 dz +
            # b1 + g1 Y' and Y' = a2 W_l^T + sbias[b] (the stored pre-BN output),
            #   dA2 = dz (diag(a1) W_l) + a2 H + cvec[b],  H = W_l^T diag(g1) W_l,
            #   dW_l = diag(a1) dz^T a2 + b1 (x) S + diag(g1) (W_l G2 + sum_b sbias[b] (x) S_b)
            # (G2 = a2^T a2, S_b = per-scene column sums of a2), so bn_seg1's Y' is not read
            p2 = sv.bn["bn2"]
            Ws1_r = self._rounded(Ws1)     # the W_l the forward GEMM used
            WaT = torch.empty(64, 512, dtype=self.tdt, device=dev)
            Hs1 = torch.empty(64, 64, dtype=self.tdt, device=dev)
            # no cvec output: the folded kernel forms its per-scene cvec_b itself (folded_cvec_kernel)
            L.call("pcs_bn_fold", L.ptr(Ws1_r), 512, 64, Ws1.shape[1], L.ptr(a1), L.ptr(b1), L.ptr(g1), self.dt,
                   L.ptr(WaT), None, L.ptr(Hs1), s)
            fa = L.WgradArgs(num_scenes=B, scene_rows=N, Cout=512, Cin=64, dtype=self.dt,
                             splits_per_scene=0, dy_mode=L.PRO_RAW, x_mode=L.PRO_BNRELU,
                             x_keep_scale=1.0, dW=L.ptr(G("seg_conv1.weight")), ldw=Ws1.shape[1],
                             flags=self.flags, dZ=L.ptr(dz_s1), alpha=L.ptr(a1),
                             beta=L.ptr(b1), gamma=L.ptr(g1), X=L.ptr(ys["conv2"]), s=L.ptr(p2.scale),
                             t=L.ptr(p2.shift))
            nbytes = L.load().pcs_dgrad_wgrad_folded_workspace(ct.byref(fa))
            if nbytes < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            ws1 = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            fa.partial = ws1.data_ptr()
            self._launch("dgrad+wgrad:seg_conv1", "pcs_dgrad_wgrad_folded", ct.byref(fa), L.ptr(WaT), L.ptr(Hs1),
                         L.ptr(Ws1_r), L.ptr(sv.sbias_s1), L.ptr(dA2), s)
            keepalive.append((ws1, Ws1_r, WaT, Hs1))
        else:
            self._gemm(B, N, 512, 64, L.PRO_BWD, L.EPI_RAW, dz_s1, wc["seg_conv1"][1], dA2,
                       A2=ys["seg_conv1"], pa=a1, pb=b1, pc=g1, tag="dgrad:seg_conv1")
            wgrad("seg_conv1", "bn_seg1", 64, 512, dz_s1, ys["seg_conv1"], "conv2", "bn2", ldw=Ws1.shape[1])

        bucket("seg")

        # global_feat input gradient in folded form (P:113 at P:254): with dy_g = beta_g +
        # gamma_g * y_g + (max-pool rows) and y_g = a5 Wg^T,
        #   dA5 = a5 H + 1 c^T + sum_b sp[b, c] Wg[c, :] at the row am[b, c],
        # H = Wg^T diag(gamma_g) Wg, c = Wg^T beta_g (pcs_bn_fold); the epilogue masks with
        # a5 > 0 (bn5's ReLU) and sums S1 = sum dz5; S2 comes from R = dz5^T a4 below.
        a5 = ys["a5"]
        Wg = P["global_feat.weight"]
        # the W the forward GEMM used (see pcs_round_weight; fp8: the dequantized e4m3 rows)
        if sv.gram5 is not None:
            Wg_r = sv.wg_eff
        else:
            Wg_r = wc["global_feat_fp8"][2] if self.fp8 else self._rounded(Wg)
        cvec = torch.empty(1024, dtype=torch.float32, device=dev)
        if self.fp8:
            # H in fp32, then e4m3 rows with one scale each (H is symmetric: row n = column n)
            Hf = torch.empty(1024, 1024, dtype=torch.float32, device=dev)
            L.call("pcs_bn_fold", L.ptr(Wg_r), 1024, 1024, Wg_r.shape[1], None, L.ptr(bg), L.ptr(gg), L.F32,
                   None, L.ptr(cvec), L.ptr(Hf), s)
            Hq, hsc, _ = self._quant_fp8(Hf)
            Hg = (Hf, Hq, hsc)
        else:
            Hg = self._empty(1024, 1024, device=dev)
            L.call("pcs_bn_fold", L.ptr(Wg_r), 1024, 1024, Wg.shape[1], None, L.ptr(bg), L.ptr(gg), self.dt,
                   None, L.ptr(cvec), L.ptr(Hg), s)
        pc5 = sv.bn["bn5"]
        cps5, _ = self.geometry(B, N, 1024, 1024, L.PRO_RAW, L.EPI_DGRAD)
        st5 = torch.empty(B * cps5, 1024, 2, dtype=torch.float32, device=dev)
        if self.fp8:
            self._gemm(B, N, 1024, 1024, L.PRO_RAW, L.EPI_DGRAD, a5, Hg[1], bufB, bias=cvec, Yp=a5,
                       w_scale=Hg[2], extra_flags=L.FLAG_AW_FP8, stats=st5, tag="dgrad:global_feat")
            L.call("pcs_pool_rows_add", L.ptr(bufB), self.dt, L.ptr(a5), L.FP8, B, N, 1024, L.ptr(sv.am),
                   L.ptr(sp), L.ptr(Wg_r), Wg_r.shape[1], 1024, L.ptr(st5), cps5, s)
        elif self.dt == L.BF16 and not (self.flags & (L.FLAG_GENERIC | L.FLAG_NO_GLDS)):
            # LDS-DMA kernel without the max-pool rows (no ordinary global loads in its
            # epilogue), then their sparse term (pcs_pool_rows_add); S1 in both
            self._gemm(B, N, 1024, 1024, L.PRO_RAW, L.EPI_DGRAD, a5, Hg, bufB, bias=cvec, Yp=a5,
                       stats=st5, tag="dgrad:global_feat")
            # the max-pool rows with the W the forward GEMM used (as the fp8 branch and the
            # Gram-form weight gradient do)
            L.call("pcs_pool_rows_add", L.ptr(bufB), self.dt, L.ptr(a5), self.dt, B, N, 1024, L.ptr(sv.am),
                   L.ptr(sp), L.ptr(Wg_r), Wg_r.shape[1], 1024, L.ptr(st5), cps5, s)
        else:
            # the max-pool rows with the W the forward GEMM used (fp32: the same tensor)
            self._gemm(B, N, 1024, 1024, L.PRO_RAW, L.EPI_DGRAD, a5, Hg, bufB, bias=cvec, Yp=a5,
                       pool_idx=sv.am, pool_coef=sp, pool_w=Wg_r, pool_ldw=Wg_r.shape[1], pool_c=1024,
                       stats=st5, tag="dgrad:global_feat")
        dz5 = bufB
        if self.perturb is not None and "dz5" in self.perturb:
            c0, c1, scale = self.perturb["dz5"]
            dz5.view(M, 1024)[:, c0:c1].mul_(scale)
        if self.capture is not None:
            self.capture.update(dz5=dz5.view(M, 1024).clone(), a5=a5, H=Hg, cvec=cvec, am=sv.am.clone(),
                                sp=sp.clone(), Wg_r=Wg_r)
        # global_feat weight gradient from the Gram of a5: the symmetric a5^T a5 (upper tiles)
        # + an O(C^3) assemble instead of the M x 1024 x 1024 GEMM
        ones = torch.ones(1024, dtype=torch.float32, device=dev)
        zeros = torch.zeros(1024, dtype=torch.float32, device=dev)
        gram = torch.empty(1024, 1024, dtype=torch.float32, device=dev)
        if sv.gram5 is not None:
            # computed in the forward (bn_global's statistics); S = sum of the per-scene sums
            gram, Sb, ws = sv.gram5
            colsum = torch.empty(1024, dtype=torch.float32, device=dev)
            L.call("pcs_reduce_partials", L.ptr(Sb), B, 1024, 1.0, L.ptr(colsum), 1024, 1024, s)
        elif self._raw_gram() and sv.a5_colsum is not None:
            # a5 is the activation itself: LDS-DMA Gram; S from conv5's per-chunk column sums
            nbytes = L.load().pcs_gram_raw_workspace(M, 1024)
            if nbytes < 0:
                raise L.PcsError(L.load().pcs_last_error().decode())
            ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            self._launch("wgrad:global_feat", "pcs_gram_raw", L.ptr(a5), M, 1024, self.a5_dt, L.ptr(ws), nbytes, L.ptr(gram), s)
            cs2 = torch.empty(1024, 2, dtype=torch.float32, device=dev)
            L.call("pcs_reduce_partials", L.ptr(sv.a5_colsum), sv.a5_colsum.shape[0], 2048, 1.0, L.ptr(cs2),
                   2048, 2048, s)
            colsum = cs2[:, 0].contiguous()
        else:
            colsum = torch.empty(1024, dtype=torch.float32, device=dev)
            sps = ct.c_int32(0)
            nbytes = L.load().pcs_gram_workspace(B, N, 1024, self.dt, ct.byref(sps))
            ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dev)
            self._launch("wgrad:global_feat", "pcs_gram", L.ptr(a5), L.ptr(ones), L.ptr(zeros), B, N, 1024,
                         self.dt, sps.value, L.ptr(ws), L.ptr(gram), L.ptr(colsum), s)
        self._launch("wgrad_asm:global_feat", "pcs_gram_wgrad", L.ptr(gram), L.ptr(colsum), L.ptr(Wg_r),
                     Wg.shape[1], L.ptr(bg), L.ptr(gg), L.ptr(sp), L.ptr(sv.am), L.ptr(a5),
                     L.ptr(ones), L.ptr(zeros), B, 1024, 1024, self.a5_dt, None, None,
                     L.ptr(G("global_feat.weight")), 1024, s)
        keepalive.append((Hg, cvec, ones, zeros, gram, colsum, ws, Wg_r))
        bucket("global")

        # conv5 (128 -> 1024): R = dz5^T a4 gives bn5's S2 (y5 = a4 W5^T is not stored) and
        # the alpha-term of dW5; then the folded input gradient and the Gram-form dW5:
        #   dA4 = dz5 (diag(alpha5) W5) + a4 (W5^T diag(gamma5) W5) + W5^T beta5
        #   dW5 = diag(alpha5) R + beta5 (x) colsum(a4) + diag(gamma5) W5 (a4^T a4)
        pc4 = sv.bn["bn4"]
        r5 = torch.empty(1024, 128, dtype=torch.float32, device=dev)
        keepalive.append(self._wgrad(B, N, 1024, 128, L.PRO_RAW, L.PRO_BNRELU, r5, tag="wgrad:conv5",
                                     dZ=dz5, X=ys["conv4"], s=pc4.scale, t=pc4.shift))
        if self.capture is not None:
            self.capture.update(r5=r5.clone(), y4=ys["conv4"], s4=pc4.scale, t4=pc4.shift)
        L.call("pcs_bn_s2_from_r", L.ptr(st5), B * cps5, 1024, L.ptr(r5), L.ptr(wc["conv5"][0]), self.dt,
               128, 128, L.ptr(pc5.mean), L.ptr(pc5.rstd), s)
        bn_bwd("bn5", "conv5", st5, cps5)
        al5, be5, ga5 = coefs["bn5"]
        W5 = P["conv5.weight"]
        W5_r = self._rounded(W5)
        ws_t = self._empty(128, 1024, device=dev)
        c5 = torch.empty(128, dtype=torch.float32, device=dev)
        h4 = self._empty(128, 128, device=dev)
        L.call("pcs_bn_fold", L.ptr(W5_r), 1024, 128, 128, L.ptr(al5), L.ptr(be5), L.ptr(ga5), self.dt,
               L.ptr(ws_t), L.ptr(c5), L.ptr(h4), s)
        # one pass: [dz5 | a4] [Ws ; H4] + c5 (PCS_PRO_CAT), then bn4's ReLU mask and S1 / S2
        cps4, _ = self.geometry(B, N, 1024 + 128, 128, L.PRO_CAT, L.EPI_DGRAD)
        st = torch.empty(B * cps4, 128, 2, dtype=torch.float32, device=dev)
        self._gemm(B, N, 1024 + 128, 128, L.PRO_CAT, L.EPI_DGRAD, dz5, ws_t, bufA, K1=1024, A2=ys["conv4"],
                   W2=h4, pa=pc4.scale, pb=pc4.shift, bias=c5, Yp=ys["conv4"], es=pc4.scale, et=pc4.shift,
                   emean=pc4.mean, erstd=pc4.rstd, stats=st, tag="dgrad:conv5")
        if self.capture is not None:
            self.capture.update(dz4=bufA[:M * 128].view(M, 128).clone(), ws_t=ws_t, h4=h4, c5=c5)
        g4, s4, ws4 = sv.gram4 if sv.gram4 is not None else \
            self._gram(ys["conv4"], pc4.scale, pc4.shift, B, N, 128, tag="gram:conv4")
        self._launch("wgrad_asm:conv5", "pcs_gram_wgrad", L.ptr(g4), L.ptr(s4), L.ptr(W5_r), 128, L.ptr(be5),
                     L.ptr(ga5), None, None, None, None, None, B, 1024, 128, self.dt, L.ptr(r5), L.ptr(al5),
                     L.ptr(G("conv5.weight")), 128, s)
        keepalive.append((ws_t, c5, h4, r5, g4, s4, ws4, W5_r))
        bn_bwd("bn4", "conv4", st, cps4)
        dz4 = bufA
        st, cps = dgrad_wgrad("conv4", "bn4", 64, 128, dz4, ys["conv4"], "conv3", "bn3", bufB)
        bn_bwd("bn3", "conv3", st, cps)
        dz3 = bufB
        st, cps = dgrad_wgrad("conv3", "bn3", 64, 64, dz3, ys["conv3"], "conv2", "bn2", bufA, addend=dA2)
        bn_bwd("bn2", "conv2", st, cps)
        dz2 = bufA
        st, cps = dgrad_wgrad("conv2", "bn2", 64, 64, dz2, ys["conv2"], "conv1", "bn1", bufB)
        bn_bwd("bn1", "conv1", st, cps)
        dz1 = bufB
        al, be, ga = coefs["bn1"]
        keepalive.append(self._wgrad(B, N, 64, self.input_dim, L.PRO_BWD, L.PRO_RAW, G("conv1.weight"),
                                     ldw=self.input_dim, conv1=True, tag="wgrad:conv1",
                                     dZ=dz1, Y=ys["conv1"], alpha=al, beta=be, gamma=ga, X=sv.x))
        bucket("tail")
        return hb
