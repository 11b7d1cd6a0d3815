NAME = "gf_nostore"
SRC = "gemm_glds"
EDITS = [("""          if (ok)
            // plain store: dz5 is re-read right away by conv5's backward (nt measured 1 ms slower)
            *reinterpret_cast<u32x4 *>(Cg + (rb + wm * 128 + i * 16 + lr) * Ncols + scol + 32 * q) =
                mk_u32x4(pk[2 * q][0], pk[2 * q][1], pk[2 * q + 1][0], pk[2 * q + 1][1]);""",
          """          asm volatile("" :: "v"(pk[2 * q][0]), "v"(pk[2 * q][1]), "v"(pk[2 * q + 1][0]), "v"(pk[2 * q + 1][1]));""")]
