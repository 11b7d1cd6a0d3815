# ablation (timing only): fwd_s12 without stage 2's MFMAs (x fragments still read)
NAME = "s12_nos2"
SRC = "fwd_s12"
EDITS = [("""          acc2[ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wfr[ct][kk]), xf[rt],
                                                                acc2[ct][rt], 0, 0, 0);""",
          """          acc2[ct][rt][0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, xf[rt])[0] ^ wfr[ct][kk][0]);""")]
