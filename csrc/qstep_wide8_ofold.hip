// Tuning build of the 8-wave 64-env-chunk step kernel with the Q(x) output layer folded into layer 2's
// epilogue (ST_WIDE_OFOLD, csrc/qstep_wide.hip); engine.step_variant = "ofold" (A/B only).
#define ST_WIDE_WAVES 8
#define ST_WIDE_PF_LATE 1
#define ST_WIDE_PF_AFTER_DW0 1
#define ST_WIDE_OFOLD 1
#define ST_WIDE_NS wide8_ofold
#define ST_WIDE_API(name) name##_ofold
#include "qstep_wide.hip"
