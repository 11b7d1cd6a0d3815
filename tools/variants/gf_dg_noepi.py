# ablation (timing only): global_feat input gradient without mask extraction and epilogue (the
# bare mainloop: no stores, no S1)
NAME = "gf_dg_noepi"
SRC = "gemm_glds"
EDITS = [("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 0, kt - kq0, tcur & 1);", ""),
         ("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 1, kt - kq0, tcur & 1);", ""),
         ("    if (kt != nks - 1) continue;\n",
          "    if (kt != nks - 1) continue;\n    if constexpr (MODE == MODE_DGRAD) { bias_init(acc); continue; }\n")]
