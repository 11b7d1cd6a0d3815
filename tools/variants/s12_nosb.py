# fwd_s12: no sched_barrier between the loop's parts (the compiler schedules the iteration freely)
NAME = "s12_nosb"
SRC = "fwd_s12"
EDITS = [
    ("""      stage1(st1, 0, acc1);
      __builtin_amdgcn_sched_barrier(0);""", """      stage1(st1, 0, acc1);"""),
    ("""      stage1(st1, 1, acc1);
      __builtin_amdgcn_sched_barrier(0);""", """      stage1(st1, 1, acc1);"""),
    ("""      stage1(st1, 2, acc1);
      __builtin_amdgcn_sched_barrier(0);""", """      stage1(st1, 2, acc1);"""),
    ("""      stage1(st1, 3, acc1);
      __builtin_amdgcn_sched_barrier(0);""", """      stage1(st1, 3, acc1);"""),
]
