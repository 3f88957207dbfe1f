// A/B build of csrc/qstep_ws.hip: x''s extra window values by ds_bpermute from the neighbour lane group
// instead of 5 of the 6 per-k-step 4-byte loads (21 -> 16 window load instructions per tile).
#define WS_PC_PERM 1
#define WS_NS ws_pcperm
#define WS_API(name) name##_pcperm
#include "../qstep_ws.hip"
