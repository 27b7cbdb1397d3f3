// Multi-sequence form of the persistent decode (k_decode_persist1m, B = 2..64): its
// own translation unit, so the single-sequence kernel's register allocation is the
// one it has alone.  The code is in t2s_persist1.hip under PERSIST1_MULTI.
#define PERSIST1_MULTI
#include "t2s_persist1.hip"
