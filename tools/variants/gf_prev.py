NAME = "gf_prev"
SRC = "gemm_glds"
REV = "HEAD"
EDITS = []
