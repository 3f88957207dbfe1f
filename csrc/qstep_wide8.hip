// 8-wave (two per SIMD) build of the 64-env-chunk step kernel: one 16-unit m-tile per wave,
// 256 registers per lane (csrc/qstep_wide.hip; selected with engine.step_waves = 8).
#define ST_WIDE_WAVES 8
#define ST_WIDE_PF_LATE 1
#define ST_WIDE_PF_AFTER_DW0 1   // prefetch after the pipelined dW0 strip (its fragment buffers need the registers)
#define ST_WIDE_NS wide8
#define ST_WIDE_API(name) name##_w8
#include "qstep_wide.hip"
