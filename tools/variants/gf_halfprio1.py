NAME = "gf_halfprio1"
SRC = "gemm_glds"
# static priority for one wave half (cdna_hip_programming.md T5, static form): wave half wm == 1
# at priority 1 for the whole K loop, no per-section flips (timing A/B only)
EDITS = [
    ("""  for (int qs = 0; qs < total; ++qs, kt = ka, tcur = ta, pcur = pa) {""",
     """  if (wm == 1) __builtin_amdgcn_s_setprio(1);
  for (int qs = 0; qs < total; ++qs, kt = ka, tcur = ta, pcur = pa) {"""),
]
