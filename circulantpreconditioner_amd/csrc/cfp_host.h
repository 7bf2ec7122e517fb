// cfp_host.h -- host-side helpers shared by the plan, the slab-distributed plan and the
// PETSc-interface layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <vector>

#include "cfp_internal.h"

namespace cfp {
int set_error(int code, const char* fmt, ...);
int hip_error(hipError_t e, const char* what);
std::vector<cd> host_twiddles(int n, int sign);
std::vector<cd> host_transport_symbol(i64 n);
int ilog2_exact(i64 v);
Side natural_side(int axis, const i64 n[3]);
void natural_cols(int axis, const i64 n[3], i64* ncols, i64* inner_n);
}  // namespace cfp

// internal plan option used by the real (r2c) plan, cfp_plan.hip
extern "C" int cfp_plan_set_external_x(struct cfp_plan_s* plan, int on);
