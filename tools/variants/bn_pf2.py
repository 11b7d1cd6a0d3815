# dgrad_wgrad_bn_kernel, COUT = 128 (conv4) only: two register sets of step operands in flight
# (the step loop unrolled by two, a set per parity): the loads of step s+3 issue at the end of
# step s and are staged at the end of step s+2, two steps of latency cover instead of one.
NAME = "bn_pf2"
SRC = "fused_bwd"
EDITS = [
    ("""  u32x4 rz[F::NCH_D], ry[F::NCH_D], rp[F::NCH_P], rd[ADD ? F::NCH_P : 1];
  uint32_t rm[MASK ? F::NCH_P : 1];
  auto load_step = [&](int64_t m0) {""",
     """  constexpr bool PF2 = COUT == 128;
  struct RS {
    u32x4 rz[F::NCH_D], ry[F::NCH_D], rp[F::NCH_P], rd[ADD ? F::NCH_P : 1];
    uint32_t rm[MASK ? F::NCH_P : 1];
  };
  RS sa, sb;
  auto load_step = [&](int64_t m0, RS &R) {
    auto &rz = R.rz; auto &ry = R.ry; auto &rp = R.rp; auto &rd = R.rd; auto &rm = R.rm;"""),
    ("""  auto store_step = [&](int64_t m0) {
#pragma unroll
    for (int i = 0; i < F::NCH_D; ++i) {""",
     """  auto store_step = [&](int64_t m0, const RS &R) {
    const auto &rz = R.rz; const auto &ry = R.ry; const auto &rp = R.rp; const auto &rd = R.rd; const auto &rm = R.rm;
#pragma unroll
    for (int i = 0; i < F::NCH_D; ++i) {"""),
    ("""  if (nsteps > 0) {
    load_step(lo);
    store_step(lo);
    __builtin_amdgcn_sched_barrier(0);
    load_step(lo + MS);
  }""",
     """  if (nsteps > 0) {
    load_step(lo, sa);
    store_step(lo, sa);
    __builtin_amdgcn_sched_barrier(0);
    load_step(lo + MS, sa);
    if constexpr (PF2) {
      __builtin_amdgcn_sched_barrier(0);
      load_step(lo + 2 * MS, sb);
    }
  }"""),
    ("""  for (int st = 0; st < nsteps; ++st) {
    const int64_t m0 = lo + (int64_t)st * MS;
    f32x4 accd[F::TPW_D];""",
     """  auto step_body = [&](int st, auto Par) __attribute__((always_inline)) {
    RS &R = (PF2 && decltype(Par)::value) ? sb : sa;
    const int64_t m0 = lo + (int64_t)st * MS;
    f32x4 accd[F::TPW_D];"""),
    ("""    if (st + 1 < nsteps) {
      store_step(m0 + MS);
      __builtin_amdgcn_sched_barrier(0);
      load_step(m0 + 2 * MS);
    }
    lds_barrier();
  }
""",
     """    if (st + 1 < nsteps) {
      store_step(m0 + MS, R);
      __builtin_amdgcn_sched_barrier(0);
      load_step(m0 + (PF2 ? 3 : 2) * MS, R);
    }
    lds_barrier();
  };
  if constexpr (PF2) {
    int st = 0;
    for (; st + 1 < nsteps; st += 2) {
      step_body(st, IC<0>{});
      step_body(st + 1, IC<1>{});
    }
    if (st < nsteps) step_body(st, IC<0>{});
  } else {
    for (int st = 0; st < nsteps; ++st) step_body(st, IC<0>{});
  }
"""),
    ("""template <int COUT, int CIN, int CB, int MS, bool MASK, bool ADD>
__global__ __launch_bounds__(THREADS) void dgrad_wgrad_bn_kernel(""",
     """template <int V> struct IC { static constexpr int value = V; };
template <int COUT, int CIN, int CB, int MS, bool MASK, bool ADD>
__global__ __launch_bounds__(THREADS) void dgrad_wgrad_bn_kernel("""),
]
