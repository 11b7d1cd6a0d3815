NAME = "gf_base"
SRC = "gemm_glds"
REV = "HEAD"
