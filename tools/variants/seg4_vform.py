# fused_seg4: the input gradient's MFMAs in the VGPR form (inline asm: dacc stays in VGPRs, so
# the 256-register dW block keeps all AGPRs and no block is parked around dacc each step); the
# epilogue's first read of dacc waits 18 cycles (XDL -> VALU read hazard, inline asm is opaque
# to hipcc's hazard recognizer)
NAME = "seg4_vform"
SRC = "fused_seg4"
EDITS = [
    ("""        dacc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[kk & 1], w, dacc[ct], 0, 0, 0);""",
     """        if constexpr (kk == 0)   // (VALU zeroing of dacc -> MFMA srcC: 2 wait states)
          asm volatile("s_nop 2\\n\\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(dacc[ct]) : "v"(bq[kk & 1]), "v"(w));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(dacc[ct]) : "v"(bq[kk & 1]), "v"(w));"""),
    ("""    // ---- epilogue of step t: masks, S1 / S2, x^T and v^T into the wave's tiles""",
     """    asm volatile("s_nop 7\\n\\ts_nop 7\\n\\ts_nop 3" : "+v"(dacc[0]), "+v"(dacc[1]), "+v"(dacc[2]), "+v"(dacc[3]));
    // ---- epilogue of step t: masks, S1 / S2, x^T and v^T into the wave's tiles"""),
]
