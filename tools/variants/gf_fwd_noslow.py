# timing only, micro-bench (tools/bench_gf.py) ONLY: the pool partials keep their sentinels (argmax = INT_MAX), which the step's pool kernels would use as row indices -- never run a training step on this build
# ablation (timing only): the forward's max-pool fast path only (the slow path never runs)
NAME = "gf_fwd_noslow"
SRC = "gemm_glds"
EDITS = [("""            if (__builtin_amdgcn_ballot_w64((beat >> j) & 1u) == 0) continue;   // uniform""",
          """            if (__builtin_amdgcn_ballot_w64((beat >> j) & 1u) != 2) continue;   // (never the slow path)""")]
