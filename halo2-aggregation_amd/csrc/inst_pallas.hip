// inst_pallas.hip -- PallasCurve instantiation of the MSM engine.
#include "accum_engine.hpp"
PM_DEFINE_CURVE_OPS(pm::PallasCurve, kPallasOps)
