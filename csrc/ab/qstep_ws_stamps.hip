// Debug build of csrc/qstep_ws.hip with s_memtime stamps per phase of data wave 0 of workgroup 0
// (tools/stamp_qstep.py --kernel ws; gradient-wave stamps: csrc/qstep_ws_gstamps.hip):
// st_qstep_ws_launch_stamps, same contract.  Kept out of the production build: the stamp code costs the
// 256-register kernel its last free registers (and with them the price prefetch's latency cover).
#define WS_STAMPS 1
#define WS_PD1 6   // (production reads 10 ahead; at 10 the stamp code spills)
#define WS_NS ws_stamps
#define WS_API(name) name##_stamps
#include "../qstep_ws.hip"
