// Experiment build of csrc/conv_h3.hip with per-block phase timestamps in
// the row-band kernels (H3_PHASE_TIMING): scripts/h3_phase.py loads this
// library next to librnb_kernels.so and routes rnb_conv_h3r_launch here.
#define H3_PHASE_TIMING 1
#include "../conv_h3.hip"

extern "C" {
// the split-K reduce lives in conv_x6.hip; the row-band kernels never call it
int rnb_x6d_splitk_reduce(const ConvF32Params*, const X6DStats*, hipStream_t) { return -99; }

int rnb_h3_phase_set(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(h3_phase_buf), &buf, sizeof(buf));
}
}
