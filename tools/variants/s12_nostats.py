# ablation (timing only): fwd_s12 without Y2's statistics accumulation
NAME = "s12_nostats"
SRC = "fwd_s12"
EDITS = [("""          *reinterpret_cast<f32x4 *>(ssp + 16 * ct) += sv;
          *reinterpret_cast<f32x4 *>(sqp + 16 * ct) += qv;""", "")]
