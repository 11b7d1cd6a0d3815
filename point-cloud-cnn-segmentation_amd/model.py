"""Drop-in ``PointNetSegmentation`` (reference: point_cloud_segmentation.py:65-133).

Same constructor ``(num_classes, input_dim=4)``, same submodule names and registration
order (10 Conv1d(k=1), 9 BatchNorm1d, Dropout(0.3)) and therefore the same 65-key
``state_dict`` / ``best_model.pth`` layout; ``forward(x[B,N,4]) -> logits[B,N,C]``.
``.train()`` / ``.eval()`` switch BatchNorm batch statistics (with running-stat updates)
and dropout exactly as nn.BatchNorm1d / nn.Dropout do.

The forward/backward run in the HIP kernels of libpcs.so via :class:`engine.Engine`
(wrapped in a ``torch.autograd.Function`` so a standard
``loss = CrossEntropyLoss(...)(out.view(-1,C), y); loss.backward(); opt.step()`` loop
works unchanged).  There is no CPU path: calling the model on a CPU tensor raises.
"""
from __future__ import annotations

import threading

import torch
import torch.nn as nn

from . import _lib as L
from .engine import BNS, FLAT_EXTRA, Engine, check_dims, flat_offsets, param_layout


class _DropoutState:
    """Per-module (per-replica) dropout state: replayed keep masks and the Philox seed stream.

    nn.DataParallel (P:209-211) replicates the module every forward by shallow-copying its
    ``__dict__`` (torch/nn/parallel/replicate.py) and runs the replicas in one thread per GPU
    (parallel_apply.py), so anything mutable on the module would be shared between threads.
    ``PointNetSegmentation._replicate_for_data_parallel`` gives every replica its own state,
    seeded from the base module's stream (under its lock, in replica order)."""

    def __init__(self, seed: int):
        self.lock = threading.Lock()
        self.gen = torch.Generator().manual_seed(seed)
        self.masks = None

    def next_seed(self) -> int:
        with self.lock:
            return int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())

    def take_masks(self):
        with self.lock:
            m, self.masks = self.masks, None
            return m


class _PointNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        eng = module._engine()
        P = module._param_dict()
        bufs = module._buffer_dict()
        train = module.training
        masks = module._take_dropout_masks() if train else None
        seed = module._next_seed() if train and masks is None else 0
        sv = eng.forward(P, bufs, x, train=train, masks=masks, seed=seed)
        if train:
            for bn, _ in BNS:
                getattr(module, bn).num_batches_tracked.add_(1)
        ctx.sv = sv
        ctx.module = module
        return sv.logits

    @staticmethod
    def backward(ctx, dlogits):
        module, sv = ctx.module, ctx.sv
        eng = module._engine()
        P = module._param_dict()
        gflat = torch.empty(eng.total_params, dtype=torch.float32, device=dlogits.device)
        eng.backward(P, sv, gflat, dlogits=dlogits)
        grads = []
        for name, shape in eng.layout:
            off = eng.offsets[name]
            grads.append(gflat[off:off + eng.numel[name]].view(shape))
        ctx.sv = None
        return (None, None, *grads)


class PointNetSegmentation(nn.Module):
    """MI355X-native PointNetSegmentation (P:65-133).

    ``compute_dtype``: ``"fp32"`` (default; exact-f32 MFMA, parity with the reference's
    fp32 CPU path), ``"bf16"`` (bf16 MFMA, fp32 accumulation and BN statistics) or ``"fp8"``
    (the bf16 path with the 1024-wide layer in e4m3: conv5 stores a5 as fp8 and global_feat's
    forward, input gradient and Gram run on MX-scaled fp8 MFMA with per-row E8M0 weight
    scales; fp32 accumulation and BN statistics throughout).

    ``eval_trunk`` (bf16 / fp8 only): precision of the EVAL forward's narrow trunk conv1..conv4.
    ``"fp32"`` (default) stores and computes it in fp32 and feeds conv5 a 16-bit split of a4:
    with trained weights, bf16 storage there moves mIoU by more than the north star's 1e-3
    (DESIGN.md section 4).  ``"bf16"`` keeps the eval forward on the training step's bf16
    storage.  Training always uses the compute dtype throughout.

    ``dropout_draw``: ``"paired"`` (default, the bench path: elements 2k and 2k + 1 share a
    byte pair of their 16-bit uniforms, each keep bit exactly Bernoulli(0.7), pair correlation
    0.0022) or ``"independent"`` (i.i.d. keep bits as nn.Dropout, P:96, for parity runs; twice
    the Philox work).
    """

    def __init__(self, num_classes, input_dim=4, *, compute_dtype: str = "fp32", eval_trunk: str = "fp32",
                 dropout_draw: str = "paired"):
        super().__init__()
        # Point-wise MLPs for feature extraction (P:70-74)
        self.conv1 = nn.Conv1d(input_dim, 64, 1)
        self.conv2 = nn.Conv1d(64, 64, 1)
        self.conv3 = nn.Conv1d(64, 64, 1)
        self.conv4 = nn.Conv1d(64, 128, 1)
        self.conv5 = nn.Conv1d(128, 1024, 1)
        self.global_feat = nn.Conv1d(1024, 1024, 1)            # P:77
        self.seg_conv1 = nn.Conv1d(1088, 512, 1)               # P:80-83
        self.seg_conv2 = nn.Conv1d(512, 256, 1)
        self.seg_conv3 = nn.Conv1d(256, 128, 1)
        self.seg_conv4 = nn.Conv1d(128, num_classes, 1)
        self.bn1 = nn.BatchNorm1d(64)                          # P:86-94
        self.bn2 = nn.BatchNorm1d(64)
        self.bn3 = nn.BatchNorm1d(64)
        self.bn4 = nn.BatchNorm1d(128)
        self.bn5 = nn.BatchNorm1d(1024)
        self.bn_global = nn.BatchNorm1d(1024)
        self.bn_seg1 = nn.BatchNorm1d(512)
        self.bn_seg2 = nn.BatchNorm1d(256)
        self.bn_seg3 = nn.BatchNorm1d(128)
        self.dropout = nn.Dropout(0.3)                         # P:96
        self.num_classes = num_classes
        self.input_dim = input_dim
        self.compute_dtype = compute_dtype
        self.eval_trunk = eval_trunk
        if dropout_draw not in ("paired", "independent"):
            raise ValueError(f"dropout_draw must be 'paired' or 'independent', got {dropout_draw!r}")
        self.dropout_draw = dropout_draw
        check_dims(num_classes, input_dim)   # fail at construction, not at the first forward
        # created lazily (it loads libpcs.so); it holds no per-call state (only a geometry
        # cache), so DataParallel replicas may share it
        self._eng = None
        self._dstate = _DropoutState(0x5eed)
        self._pnames = [n for n, _ in param_layout(num_classes, input_dim)]

    # ---------------------------------------------------------------- internals
    def _engine(self) -> Engine:
        if (self._eng is None or self._eng.dtype != self.compute_dtype
                or self._eng.eval_trunk != self.eval_trunk):
            self._eng = Engine(self.num_classes, self.compute_dtype, self.input_dim, self.eval_trunk)
        self._eng.dropout_draw = self.dropout_draw
        return self._eng

    def _params(self):
        """The parameters in registration order, by attribute: on a DataParallel replica they
        are the broadcast copies that replicate() sets as plain attributes (its
        ``_parameters`` is empty), so named_parameters() would see none of them."""
        out = []
        for n in self._pnames:
            mod, attr = n.split(".")
            out.append(getattr(getattr(self, mod), attr))
        return out

    def _param_dict(self):
        return dict(zip(self._pnames, self._params()))

    _flat_extra = FLAT_EXTRA   # gradient-buffer tail used by the fused data-parallel step

    def _flat_offsets(self):
        """Parameter offsets in the flat fp32 buffers (engine.flat_layout: bucket order)."""
        return flat_offsets(self.num_classes, self.input_dim)[0]

    def _buffer_dict(self):
        return {n: b for n, b in self.named_buffers()}

    def _next_seed(self):
        return self._dstate.next_seed()

    def _replicate_for_data_parallel(self):
        replica = super()._replicate_for_data_parallel()
        replica._dstate = _DropoutState(self._next_seed())
        return replica

    def set_dropout_masks(self, bits1, bits2):
        """Replay dropout keep masks in the next train forward (tests / reference parity).

        bits1: uint8 [B*N, 64] (512 channels after bn_seg1, P:124), bits2: uint8 [B*N, 32]
        (256 channels after bn_seg2, P:126); bit i of byte j = channel 8j+i.
        """
        with self._dstate.lock:
            self._dstate.masks = (bits1.contiguous(), bits2.contiguous())

    def _take_dropout_masks(self):
        return self._dstate.take_masks()

    def seed_dropout(self, seed: int):
        with self._dstate.lock:
            self._dstate.gen.manual_seed(seed)

    # ---------------------------------------------------------------- API
    def forward(self, x):
        """x: (batch_size, max_points, 4) -> logits (batch_size, max_points, num_classes)."""
        if x.dim() != 3 or x.shape[-1] != self.input_dim:
            raise ValueError(f"expected x of shape (B, N, {self.input_dim}), got {tuple(x.shape)}")
        if not x.is_cuda:
            raise RuntimeError("pcs_amd.PointNetSegmentation runs on a HIP device only; "
                               "move the model and inputs with .to('cuda')")
        return _PointNetFunction.apply(x, self, *self._params())


def load_reference_checkpoint(path, map_location="cpu"):
    """Load a reference ``best_model.pth`` (P:373-382) safely (weights_only=True).

    Returns (state_dict without any 'module.' prefix, checkpoint dict).  The prefix
    handling mirrors P:409-428.
    """
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    sd = ckpt["model_state_dict"] if "model_state_dict" in ckpt else ckpt
    if any(k.startswith("module.") for k in sd):
        sd = {k.replace("module.", "", 1): v for k, v in sd.items()}
    return sd, ckpt
