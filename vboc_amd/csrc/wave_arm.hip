// wave_arm.hip - the UR5 arm's wave solver (coop_arm.h) as its own translation unit, compiled at -O1 and
// linked into libvboc_amd.so next to vboc_solver.hip (-O3).  See DESIGN.md section 13.
#define VBOC_ARM_TU
#include "vboc_solver.hip"
