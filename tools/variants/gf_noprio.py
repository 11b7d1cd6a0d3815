NAME = "gf_noprio"
SRC = "gemm_glds"
# no s_setprio around the MFMA sections (timing A/B only)
EDITS = [
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(0, 0);
    __builtin_amdgcn_s_setprio(0);""", """    mfma_quad(0, 0);"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(0, 2);
    __builtin_amdgcn_s_setprio(0);""", """    mfma_quad(0, 2);"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(4, 0);
    __builtin_amdgcn_s_setprio(0);""", """    mfma_quad(4, 0);"""),
    ("""    __builtin_amdgcn_s_setprio(1);
    mfma_quad(4, 2);
    __builtin_amdgcn_s_setprio(0);""", """    mfma_quad(4, 2);"""),
]
