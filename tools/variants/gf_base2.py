NAME = "gf_base2"
SRC = "gemm_glds"
REV = "HEAD"
