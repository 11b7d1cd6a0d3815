# ablation (timing only): fwd_s12 writes the rounded Y1 as x (no bn_seg1 / ReLU / keep)
NAME = "s12_nox"
SRC = "fwd_s12"
EDITS = [("""      uint2 xo = make_uint2(pack2bf(x0, x1), pack2bf(x2, x3));""",
          """      uint2 xo = make_uint2(pk[rt][0], pk[rt][1]);"""),
         ("""        xo.x &= m.x;
        xo.y &= m.y;""", "")]
