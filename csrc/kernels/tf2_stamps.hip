// tf2.hip with per-phase s_memrealtime timers compiled in (diagnostics: tools/phase_profile.py --split 4).
// afl_tf2_train dispatches here when the caller passes a stamps buffer, so the production kernel carries
// no timer code or registers.
#define TF2_STAMPS 1
#include "tf2.hip"
