// Tuning build of the 8-wave 64-env-chunk step kernel with XOR-swizzled, unpadded weight images
// (ST_WIDE_WSWZ, csrc/qstep_wide.hip); engine.step_variant = "wswz".
#define ST_WIDE_WAVES 8
#define ST_WIDE_PF_LATE 1
#define ST_WIDE_PF_AFTER_DW0 1
#define ST_WIDE_WSWZ 1
#define ST_WIDE_NS wide8_wswz
#define ST_WIDE_API(name) name##_wswz
#include "qstep_wide.hip"
