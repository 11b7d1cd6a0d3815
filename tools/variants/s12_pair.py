# fwd_s12: stage 1 two 16-column tiles at a time, sharing the a2 fragments (half the a2 LDS reads)
NAME = "s12_pair"
SRC = "fwd_s12"
EDITS = [
    ("""  // its epilogue: scene bias, round into pk""",
     """  auto stage1p = [&](const char *st, int hq, f32x4 (&ap)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      ap[c][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      ap[c][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bf[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        bf[rt] = *reinterpret_cast<const bf16x8 *>(st + (16 * rt + l16) * ROW1 + (((4 * kk + g) ^ fa) << 4));
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16x8 af = *reinterpret_cast<const bf16x8 *>(lds + OFF_W1 + (64 * w + 16 * (2 * hq + c) + l16) * ROW1 +
                                                            (((4 * kk + g) ^ fa) << 4));
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) ap[c][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[rt], ap[c][rt], 0, 0, 0);
      }
    }
  };
  // its epilogue: scene bias, round into pk"""),
    ("""      f32x4 acc1[2];
      uint32_t pa[2][2], pb[2][2];
      stage2(xr, 0, 3, acc2);
      stage1(st1, 0, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 3, 3, acc2);
      epi1(st1, xw, 0, acc1, pa);
      stage1(st1, 1, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 6, 3, acc2);
      epi1(st1, xw, 1, acc1, pb);
      store1(pa, pb, 0, out1);
      stage1(st1, 2, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 9, 3, acc2);
      epi1(st1, xw, 2, acc1, pa);
      stage1(st1, 3, acc1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 12, 4, acc2);
      epi1(st1, xw, 3, acc1, pb);
      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);""",
     """      f32x4 ap[2][2];
      uint32_t pa[2][2], pb[2][2];
      stage2(xr, 0, 4, acc2);
      stage1p(st1, 0, ap);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 4, 4, acc2);
      epi1(st1, xw, 0, ap[0], pa);
      epi1(st1, xw, 1, ap[1], pb);
      store1(pa, pb, 0, out1);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 8, 4, acc2);
      stage1p(st1, 1, ap);
      __builtin_amdgcn_sched_barrier(0);
      stage2(xr, 12, 4, acc2);
      epi1(st1, xw, 2, ap[0], pa);
      epi1(st1, xw, 3, ap[1], pb);
      store1(pa, pb, 1, out1);
      __builtin_amdgcn_sched_barrier(0);"""),
]
