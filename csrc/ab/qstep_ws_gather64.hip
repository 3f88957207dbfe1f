// A/B build of csrc/qstep_ws.hip: the window gather's k order permuted (slot_col) so that each of the
// 12 window load instructions per tile covers one 64-byte run per env (instead of 4 x 16 bytes at a
// 32-byte stride), x''s shifted values by ds_bpermute from the next lane group: 16 window loads per tile.
#define WS_GATHER64 1
#define WS_NS ws_gather64
#define WS_API(name) name##_gather64
#include "../qstep_ws.hip"
