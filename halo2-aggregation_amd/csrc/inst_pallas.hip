// inst_pallas.hip -- PallasCurve instantiation of the MSM engine.
#include "engine.hpp"
PM_DEFINE_CURVE_OPS(pm::PallasCurve, kPallasOps)
