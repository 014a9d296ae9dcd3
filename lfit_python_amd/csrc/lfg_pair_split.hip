// lfg_pair_split.hip -- k_pair's fold and LONG instantiations, compiled from
// lfg.hip's own source with -mllvm -disable-machine-licm (why: the comment
// at lfg_pair_launch_split in lfg.hip).  Only the kernels this launcher
// instantiates are taken from here; lfg.hip's C ABI is compiled out.
#define LFG_NOLICM_TU 1
#include "lfg.hip"

#ifndef LFG_ONE_TU
void lfg_pair_launch_split(int variant, unsigned grid, hipStream_t st, const void* args)
{
    const PairArgs& A = *static_cast<const PairArgs*>(args);
    if (variant == PAIR_SPLIT_LONG) hipLaunchKernelGGL((k_pair<false, false, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
    else if (variant == PAIR_SPLIT_FOLD) hipLaunchKernelGGL((k_pair<false, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
    else hipLaunchKernelGGL((k_pair<false, true, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
}
#endif
