// Debug build of csrc/qstep_ws.hip: s_memtime stamps of gradient wave 0 of workgroup 0 per ring slot
// (tools/stamp_qstep.py --kernel ws; the data-wave stamps are csrc/qstep_ws_stamps.hip -- one kind of
// wave per build, so neither build's stamps cost the other kind its registers).
// st_qstep_ws_launch_gstamps (engine.step_variant = "gstamps" with step_kernel "ws").
#define WS_STAMPS 2
#define WS_NS ws_gstamps
#define WS_API(name) name##_gstamps
#include "../qstep_ws.hip"
