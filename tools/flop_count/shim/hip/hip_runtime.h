// host shim for tools/flop_count: the HIP qualifiers and the two gfx950
// builtins lfg_device.hpp uses, mapped onto counting host functions
#pragma once
#define __device__
#define __host__
#define __global__
#define __constant__
#define __forceinline__ inline
#define __noinline__
#define __builtin_amdgcn_rsq(x) lfg_rsq(x)
#define __builtin_amdgcn_rcp(x) lfg_rcp(x)
using std::max;  // integer min/max of the device code (HIP provides them on the device; count.cpp includes <algorithm> first)
using std::min;
