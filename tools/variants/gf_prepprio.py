NAME = "gf_prepprio"
SRC = "gemm_glds"
# the preparation (reads, DMA issue, waits) at priority 1, the MFMA sections at 0 (timing A/B only)
EDITS = [
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier_raw();""", """    __builtin_amdgcn_s_setprio(0);
    mfma_quad(0, 0);
    __builtin_amdgcn_s_setprio(1);
    barrier_raw();"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(0, 2);
    __builtin_amdgcn_s_setprio(0);
    barrier_raw();""", """    __builtin_amdgcn_s_setprio(0);
    mfma_quad(0, 2);
    __builtin_amdgcn_s_setprio(1);
    barrier_raw();"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(4, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier_raw();""", """    __builtin_amdgcn_s_setprio(0);
    mfma_quad(4, 0);
    __builtin_amdgcn_s_setprio(1);
    barrier_raw();"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(4, 2);
    __builtin_amdgcn_s_setprio(0);
    barrier_raw();""", """    __builtin_amdgcn_s_setprio(0);
    mfma_quad(4, 2);
    __builtin_amdgcn_s_setprio(1);
    barrier_raw();"""),
]
