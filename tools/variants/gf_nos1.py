NAME = "gf_nos1"
SRC = "gemm_glds"
EDITS = [("            s1[j][r] += v[r];\n", ""),
         ("      if (do_stats) run[cme].x += S1;", "      (void)S1;")]
