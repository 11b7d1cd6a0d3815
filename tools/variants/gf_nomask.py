NAME = "gf_nomask"
SRC = "gemm_glds"
EDITS = [("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 0, kt - kq0, tcur & 1);", ""),
         ("if (MODE == MODE_DGRAD && (unsigned)(kt - kq0) < NKQ) extract_mask(buf, 1, kt - kq0, tcur & 1);", ""),
         ("const int word = ok ? (int)((j < 2 ? mw.x : mw.y) >> ((j & 1) * 16 + 4 * lg)) : 0;",
          "const int word = ok ? -1 : 0; (void)mw;")]
