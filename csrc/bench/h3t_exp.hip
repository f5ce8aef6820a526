// Experiment builds of the temporal frame-band kernel (conv_h3t_kernel) with
// parts of the work removed (H3T_EXP, see conv_h3.hip): scripts/h3t_exp.py
// compiles this file once per variant and routes rnb_conv_h3t_launch here.
#ifndef H3T_EXP
#error "build with -DH3T_EXP=<variant>"
#endif
#include "../conv_h3.hip"

extern "C" {
// the split-K reduce lives in conv_x6.hip; the band kernels never call it
int rnb_x6d_splitk_reduce(const ConvF32Params*, const X6DStats*, hipStream_t) { return -99; }
}
