// host shim for cpu_baseline/lfg_cpu.cpp: the HIP qualifiers and the two
// gfx950 builtins lfit_python_amd/csrc/lfg_device.hpp uses, as host code
// (v_rcp_f64 / v_rsq_f64 -> the exact IEEE operations)
#pragma once
#include <algorithm>
#include <cmath>
#define __device__
#define __host__
#define __global__
#define __constant__
#define __forceinline__ inline
#define __noinline__
#define __builtin_amdgcn_rsq(x) (1.0 / std::sqrt(x))
#define __builtin_amdgcn_rcp(x) (1.0 / (x))
using std::max;  // the device code's integer min / max
using std::min;
inline double rsqrt(double x) { return 1.0 / std::sqrt(x); }
inline float rsqrtf(float x) { return 1.0f / std::sqrt(x); }
