# ablation (timing only): global_feat input gradient with no mask extraction and an epilogue that
# only keeps the accumulators alive (the MFMAs stay; no stores, no S1)
NAME = "gf_dg_noepi2"
SRC = "gemm_glds"
EDITS = [("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 0, kt - kq0, tcur & 1);", ""),
         ("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 1, kt - kq0, tcur & 1);", ""),
         ("    if (kt != nks - 1) continue;\n",
          """    if (kt != nks - 1) continue;
    if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
      bias_init(acc);
      continue;
    }
""")]
