// Diagnostic build of rnn2.hip with per-phase timers (tools/phase_profile.py --model RNNModel)
#define RNN2_STAMPS 1
#include "rnn2.hip"
