// A/B variant of t2s_persistm.hip (tools/build_alt.sh): weight loads after the gathers
#define PERSISTM_LATE_W 1
#include "t2s_persistm.hip"
