# ablation (timing only): fwd_s12 without applying the keep bits
NAME = "s12_nomask"
SRC = "fwd_s12"
EDITS = [("""        xo.x &= m.x;
        xo.y &= m.y;""", "")]
