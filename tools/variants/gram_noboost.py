NAME = "gram_noboost"
SRC = "gram_glds"
# no priority boost around the Gram's MFMA sections (the base priority above the draw stays;
# timing A/B only, after the global_feat GEMMs gained from dropping theirs in r06)
EDITS = [(f"""    __builtin_amdgcn_s_setprio(1 + GG_PRIO);
    mfma_quad({a}, {b});
    __builtin_amdgcn_s_setprio(GG_PRIO);""", f"""    mfma_quad({a}, {b});""") for a, b in ((0, 0), (0, 2), (4, 0), (4, 2))]
