// inst_vesta.hip -- VestaCurve instantiation of the MSM engine.
#include "accum_engine.hpp"
PM_DEFINE_CURVE_OPS(pm::VestaCurve, kVestaOps)
