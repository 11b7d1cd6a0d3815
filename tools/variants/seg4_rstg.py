# fused_seg4, COUT = 128 only: the step pieces come through registers (raw buffer loads ->
# ds_write) instead of LDS-DMA.  Loads of step t+3 issue at the end of step t into one register
# set, which the end of step t+1 writes into step t+3's stage (one step of latency cover);
# hipcc tracks the loads, so the counted DMA waits go away for this shape.
NAME = "seg4_rstg"
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
  u32x4 rg[F::NPW];
  uint32_t rgb = 0;
  auto load_piece = [&](auto Ic, int s) __attribute__((always_inline)) {
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
  auto write_set = [&](int sidx) __attribute__((always_inline)) {
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
      sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, s); });
      write_set(s);
    }
    sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, 2); });
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
      write_set(sc + 2 >= NST ? sc + 2 - NST : sc + 2);   // step t+2 (loaded at the end of step t-1)
      sfor<F::VM_STEP>([&](auto Ic) __attribute__((always_inline)) { load_piece(Ic, t + 3); });
    }
    sd = sc;
    sc = sn;"""),
]
