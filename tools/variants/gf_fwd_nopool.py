# ablation (timing only): global_feat forward without its max-pool epilogue (the bare mainloop)
NAME = "gf_fwd_nopool"
SRC = "gemm_glds"
EDITS = [("""        if (do_pool) {
          // only the extremum""", """        if (false) {
          // only the extremum""")]
