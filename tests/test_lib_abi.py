"""CPU-side checks of the C ABI: the library loads and exports every declared symbol."""
import ctypes as ct
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pcs.h")
LIB = os.path.join(REPO, "point-cloud-cnn-segmentation_amd", "csrc", "libpcs.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared_functions()
    for n in ["pcs_gemm", "pcs_wgrad", "pcs_head", "pcs_adam", "pcs_bn_fwd_finalize",
              "pcs_bn_bwd_finalize", "pcs_pool_finalize", "pcs_pool_bwd", "pcs_dropout_bits"]:
        assert n in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (same HIP runtime as the product path)
    lib = ct.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    lib.pcs_abi_version.restype = ct.c_int
    hdr = open(os.path.join(REPO, "include", "pcs.h")).read()
    want = int(re.search(r"#define PCS_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.pcs_abi_version() == want == 2
    import pcs_amd._lib as L
    assert L.ABI_VERSION == want


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_binding_signatures_cover_header():
    import pcs_amd._lib as L
    bound = {n for n, _, _ in L.SIGNATURES}
    assert set(declared_functions()) == bound


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_argument_validation_without_gpu():
    """Invalid arguments are rejected on the host, before any launch (no GPU needed)."""
    import pcs_amd._lib as L
    lib = L.load()
    a = L.GemmArgs(num_scenes=1, scene_rows=128, K=60, Ncols=64, dtype=L.BF16)
    assert lib.pcs_gemm(ct.byref(a), None) == -1000
    assert b"multiple" in lib.pcs_last_error()
    h = L.HeadArgs(num_scenes=1, scene_rows=64, Cin=128, num_classes=40)
    assert lib.pcs_head(ct.byref(h), None) == -1000
    assert lib.pcs_dropout_bits(1, 0, 16, 12, 0.3, None, None) == -1000


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_geometry_is_scene_aligned():
    import pcs_amd._lib as L
    lib = L.load()
    for N, B in [(4096, 4), (3000, 3), (2097152, 4), (1, 1), (129, 2)]:
        a = L.GemmArgs(num_scenes=B, scene_rows=N, K=64, Ncols=1024, dtype=L.BF16)
        rpc = lib.pcs_gemm_geometry(ct.byref(a))
        assert rpc % 128 == 0 and rpc > 0
        cps = a.chunks_per_scene
        assert (cps - 1) * rpc < N <= cps * rpc      # no empty chunk, full coverage


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_fused_dgrad_wgrad_validates_shapes_without_gpu():
    import pcs_amd._lib as L
    lib = L.load()
    a = L.WgradArgs(num_scenes=1, scene_rows=128, Cout=256, Cin=64, dtype=L.BF16, dy_mode=L.PRO_BWD,
                    x_mode=L.PRO_BNRELU)
    assert lib.pcs_dgrad_wgrad_workspace(ct.byref(a)) < 0
    a.Cout = 512
    assert lib.pcs_dgrad_wgrad_workspace(ct.byref(a)) == a.splits_per_scene * 512 * 64 * 4


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_conv3d_argument_validation_without_gpu():
    """pcs_conv3d* reject bad geometries on the host, before any launch (no GPU needed)."""
    import pcs_amd._lib as L
    lib = L.load()

    def geom(**kw):
        d = dict(B=1, Di=8, Hi=8, Wi=8, Do=8, Ho=8, Wo=8, Cin=64, Cout=64, k=3, s=1, p=1, transposed=0)
        d.update(kw)
        return L.Conv3dGeom(**d)

    ok = geom()
    assert lib.pcs_conv3d_wgrad_workspace(ct.byref(ok)) > 0
    for bad in (geom(Cin=48), geom(Cout=40), geom(Do=7), geom(k=4), geom(s=3), geom(p=3),
                geom(transposed=1, Do=9)):
        assert lib.pcs_conv3d(ct.byref(bad), 1, 1, None, 1, L.BF16, None) == -1000
    assert lib.pcs_conv3d(ct.byref(ok), 1, 1, None, 1, L.F32 + 7, None) == -1000
    assert lib.pcs_conv3d_wgrad_workspace(ct.byref(geom(Cin=40))) == -1000
    assert lib.pcs_conv3d_wgrad_workspace(ct.byref(geom(Cin=32, Cout=96))) > 0   # 32-channel tiles
    up = geom(Di=4, Hi=4, Wi=4, k=2, s=2, p=0, transposed=1)     # 4^3 -> 8^3
    assert lib.pcs_conv3d_wgrad_workspace(ct.byref(up)) > 0


def test_seg_backward_geometry_without_gpu():
    """seg_conv2 / seg_conv3 backward (pcs_dgrad_wgrad_bn): the four-wave kernel's slices
    (fused_seg4.hip: 16-row steps, one 256-column workgroup per CU)."""
    import pcs_amd._lib as L
    lib = L.load()
    for cout, cin in ((256, 512), (128, 256)):
        for flags, nblk in ((0, cin // 256),):
            a = L.GemmArgs(num_scenes=4, scene_rows=128 ** 3, K=cout, Ncols=cin, dtype=L.BF16,
                           prologue=L.PRO_BWD, epilogue=L.EPI_DGRAD, flags=flags)
            nbytes = lib.pcs_dgrad_wgrad_bn_workspace(ct.byref(a))
            cps = a.chunks_per_scene
            assert nbytes == 4 * cps * cout * cin * 4
            assert cps * 4 * nblk >= 256 and cps * 4 * nblk < 2 * 256   # about one workgroup per CU


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcs.so not built")
def test_sparse_pairs_argument_validation_without_gpu():
    """The pair-list entry points reject bad tap offsets and channel counts on the host, before
    any launch, and size their workspaces from the host tap offsets (no GPU needed)."""
    import pcs_amd._lib as L
    lib = L.load()
    assert lib.pcs_sparse_pairs_workspace(1000, 27) == ((1000 + 255) // 256 * 27 + 1) * 4
    assert lib.pcs_sparse_pairs_workspace(-1, 27) == -1000
    assert lib.pcs_sparse_pairs_workspace(10, 28) == -1000
    good = (ct.c_int64 * 28)(*([0] * 13 + [100] * 15))       # only the centre tap: 100 rows
    ta = ct.addressof(good)
    assert lib.pcs_sparse_conv_wgrad_pairs_workspace(ta, 27, 100, 64, 64) > 0
    assert lib.pcs_sparse_conv_wgrad_pairs_workspace(ta, 27, 100, 32, 64) == -1000   # Cin % 64
    # slices are divided over the 64 x 64 channel tiles: 27 taps x 2^20 pairs keep the workspace
    # near 2048 tiles' partials at every width (a fixed 2048 slices took 544 MB at 256 -> 256)
    V = 1 << 20
    full = (ct.c_int64 * 28)(*[t * V for t in range(28)])
    for ch, lim in ((64, 40 << 20), (128, 48 << 20), (256, 48 << 20)):
        nb = lib.pcs_sparse_conv_wgrad_pairs_workspace(ct.addressof(full), 27, V, ch, ch)
        assert 0 < nb <= lim, (ch, nb)
    bad = (ct.c_int64 * 28)(*([0] * 13 + [100] * 14 + [50]))   # decreasing
    assert lib.pcs_sparse_conv_wgrad_pairs_workspace(ct.addressof(bad), 27, 100, 64, 64) == -1000
    start = (ct.c_int64 * 28)(*([5] + [100] * 27))             # not starting at 0
    assert lib.pcs_sparse_conv_pairs(1, 1, ct.addressof(start), 27, 100, 1, 64, 1, 64, None, 1, 1, L.BF16, 0,
                                     None) == -1000
    assert lib.pcs_sparse_conv_pairs(1, 1, ta, 27, 100, 1, 64, 1, 48, None, 1, 1, L.BF16, 0, None) == -1000   # Cout
    assert lib.pcs_sparse_conv_pairs(1, 1, ta, 27, 100, 1, 64, 1, 64, None, None, 1, L.BF16, 0, None) == -1000   # no Z
