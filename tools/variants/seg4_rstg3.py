# seg4_rstg with two register sets (the step loop unrolled by two, a set per parity): loads of step t+4 issue
# at the end of step t, written at the end of step t+2 (two steps of latency cover).
NAME = "seg4_rstg3"
SRC = "fused_seg4"
EDITS = [
    ("""    m0_restore(keep);
  };
""",
     """    m0_restore(keep);
  };
  constexpr bool RSTG = COUT == 128;
  const __amdgpu_buffer_rsrc_t br_dz = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(dZg), 0, (int)((uint32_t)rows * ROWB), 0x00020000);
  const __amdgpu_buffer_rsrc_t br_y = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(Yg), 0, (int)((uint32_t)rows * ROWB), 0x00020000);
  const __amdgpu_buffer_rsrc_t br_yp = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(Ypg), 0, (int)((uint32_t)rows * (CIN * 2)), 0x00020000);
  const __amdgpu_buffer_rsrc_t br_mk = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(Mkg), 0, (int)((uint32_t)rows * MKROW), 0x00020000);
  u32x4 rgA[F::NPW], rgB[F::NPW];
  uint32_t rgbA = 0, rgbB = 0;
  auto load_piece = [&](auto Ic, int s, u32x4 (&rg)[F::NPW], uint32_t &rgb) __attribute__((always_inline)) {
    constexpr int i = decltype(Ic)::value;
    if constexpr (i == F::NPW)
      rgb = __builtin_amdgcn_raw_buffer_load_b32(br_mk, (int)voff[i], s * MS * MKROW, 0);
    else if constexpr (4 * i < F::NPD)
      rg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(br_dz, (int)voff[i], s * MS * ROWB, 0));
    else if constexpr (4 * i < 2 * F::NPD)
      rg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(br_y, (int)voff[i], s * MS * ROWB, 0));
    else
      rg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(br_yp, (int)voff[i], s * MS * CIN * 2, 0));
  };
  auto write_set = [&](int sidx, const u32x4 (&rg)[F::NPW], uint32_t rgb) __attribute__((always_inline)) {
    char *b = lds + sidx * F::STAGE;
#pragma unroll
    for (int i = 0; i < F::NPW; ++i) *reinterpret_cast<u32x4 *>(b + 4096 * i + wid * 1024 + lane * 16) = rg[i];
    *reinterpret_cast<uint32_t *>(b + 2 * F::DZB + F::YPB + (wid & 1) * 256 + lane * 4) = rgb;
  };
"""),
    ("""#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { dma_piece(Ic, s, s); });
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
  }
  wait_vm<2 + (NST - 2) * (F::VM_STEP + 2)>();""",
     """  if constexpr (RSTG) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, s, rgA, rgbA); });
      write_set(s, rgA, rgbA);
    }
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, 2, rgA, rgbA); });
    __builtin_amdgcn_sched_barrier(0);   // (set A older than set B, as in the loop)
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, 3, rgB, rgbB); });
  } else {
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { dma_piece(Ic, s, s); });
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
    store_rows(0xFFFFFF00u, mk_u32x4(0, 0, 0, 0));
  }
  wait_vm<2 + (NST - 2) * (F::VM_STEP + 2)>();
  }"""),
    ("""    wait_vm<2 + (NST - 3) * (F::VM_STEP + 2)>();
    barrier_lds();""",
     """    if constexpr (!RSTG) wait_vm<2 + (NST - 3) * (F::VM_STEP + 2)>();
    barrier_lds();"""),
    ("""      if constexpr (kk <= F::NPW) dma_piece(IC<kk>{}, sdma, sd);""",
     """      if constexpr (!RSTG && kk <= F::NPW) dma_piece(IC<kk>{}, sdma, sd);"""),
    ("""    sfor<F::VM_STEP - (F::KSD < F::VM_STEP ? F::KSD : F::VM_STEP)>([&](auto Ic) __attribute__((always_inline)) {
      dma_piece(IC<F::KSD + decltype(Ic)::value>{}, sdma, sd);   // (seg_conv3: 4 k-steps, 5 pieces)
    });""",
     """    if constexpr (!RSTG)
    sfor<F::VM_STEP - (F::KSD < F::VM_STEP ? F::KSD : F::VM_STEP)>([&](auto Ic) __attribute__((always_inline)) {
      dma_piece(IC<F::KSD + decltype(Ic)::value>{}, sdma, sd);   // (seg_conv3: 4 k-steps, 5 pieces)
    });"""),
    ("""    sd = sc;
    sc = sn;""",
     """    if constexpr (RSTG) {
      const int s2 = sc + 2 >= NST ? sc + 2 - NST : sc + 2;   // step t+2 (loaded at the end of step t-2)
      if constexpr (decltype(Par)::value) {
        write_set(s2, rgB, rgbB);
        sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, t + 4, rgB, rgbB); });
      } else {
        write_set(s2, rgA, rgbA);
        sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, t + 4, rgA, rgbA); });
      }
    }
    sd = sc;
    sc = sn;"""),
    ("""  for (int t = 0; t < nsteps; ++t) {""",
     """  auto step_body = [&](int t, auto Par) __attribute__((always_inline)) {"""),
    ("""  }
  wait_vm<0>();   // the clamped DMAs past the end""",
     """  };
  if constexpr (RSTG) {
    int t = 0;
    for (; t + 1 < nsteps; t += 2) {
      step_body(t, IC<0>{});
      step_body(t + 1, IC<1>{});
    }
    if (t < nsteps) step_body(t, IC<0>{});
  } else {
    for (int t = 0; t < nsteps; ++t) step_body(t, IC<0>{});
  }
  wait_vm<0>();   // the clamped DMAs past the end"""),
]
