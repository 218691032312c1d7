// inst_bn254.hip -- Bn254Curve instantiation of the MSM engine.
#include "accum_engine.hpp"
PM_DEFINE_CURVE_OPS(pm::Bn254Curve, kBn254Ops)
