// BatchNorm finalize folded into the producing conv ("BN tail"): the conv
// whose epilogue accumulates a BN's per-video fp64 sums also turns them into
// the per-video scale / shift rows the next conv applies on load, in the
// last wave of its own launch -- no bn_seg_ss_from_sums_f32_kernel dispatch
// between the two convs (a one-clip forward carried 46 of them, ~4.7 us
// each, profiles/r6_bnbreak_1clips.txt).
//
// Every wave of the launch, once its sums atomics are performed (s_waitcnt
// vmcnt(0): agent-scope fp64 atomics, done beyond the XCD's L2), adds 1 to
// the BN's ticket; the wave that brings it to `expect` (the launch's wave
// count) reads the sums with sc1 loads (L1 bypassed, no stale line: the
// atomics left none in any L2), computes scale / shift for all nseg x C
// (segment, channel) pairs with the formulas of bn_seg_ss_from_sums_f32_kernel
// and re-arms the ticket to 0 for the next launch (stream-ordered). No
// agent-scope fence: __threadfence() writes back and invalidates the XCD's L2
// in every wave that runs it -- a first build with it ran the one-clip
// forward at 4.3 ms instead of 2.3 (profiles/r6_bn_tail_threadfence.txt). The
// producer's launcher takes the tail that the host armed (rnb_bn_tail_arm)
// for the LAST launch of the conv only, so when that wave runs every sums
// atomic of the conv has been performed. Sums stay in place: the forward's
// batched running update walks and re-arms them (bn_seg_running_batched).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct BnTail {
  int* ticket;               // null: no tail (the host finalizes separately)
  int expect;                // waves of the launch that reach the tail
  int nseg, C, sums_c, rpc;  // segments (videos), channels, sums row stride, rows per clip
  const double* sums;        // [nseg][2][sums_c]
  const int* coffs;          // [nseg + 1] clip offsets
  const float* gamma;
  const float* beta;
  float eps;
  float* ss;                 // out: [nseg][2][C] (scale row, shift row)
};

// host: the armed tail for a launch of `waves` waves (disarmed on return;
// ticket null when none is armed). Defined in bn_ops.hip.
BnTail bn_tail_take(long long waves);

// sc1 load (global_load_dwordx2 ... sc1): bypasses this CU's L1
static __device__ __forceinline__ double bn_tail_load(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by every wave of a producer launch after its epilogue (all lanes
// converged; the wave's sums atomics issued).
static __device__ __forceinline__ void bn_tail_run(const BnTail& t) {
  if (t.ticket == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sums atomics: performed
  const unsigned long long live = __ballot(1);
  const int leader = __ffsll((long long)live) - 1;
  const int lane = threadIdx.x & 63;
  int old = 0;
  if (lane == leader) old = atomicAdd(t.ticket, 1);
  old = __shfl(old, leader, 64);
  if (old != t.expect - 1) return;
  const int total = t.nseg * t.C;
  for (int i0 = 0; i0 < total; i0 += 8 * 64) {
    // eight (segment, channel) pairs per lane in flight
    double a1[8], a2[8];
    int rows[8], sg[8], ch[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + lane;
      sg[u] = i < total ? i / t.C : 0;
      ch[u] = i < total ? i - sg[u] * t.C : -1;
      const double* sp = t.sums + (size_t)sg[u] * 2 * t.sums_c;
      a1[u] = ch[u] >= 0 ? bn_tail_load(sp + ch[u]) : 0.0;
      a2[u] = ch[u] >= 0 ? bn_tail_load(sp + t.sums_c + ch[u]) : 0.0;
      rows[u] = ch[u] >= 0 ? (t.coffs[sg[u] + 1] - t.coffs[sg[u]]) * t.rpc : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (ch[u] < 0) continue;
      float mu = 0.f, va = 0.f;
      if (rows[u] > 0) {
        const double m = a1[u] / (double)rows[u];
        mu = (float)m;
        va = (float)fmax(a2[u] / (double)rows[u] - m * m, 0.0);
      }
      const float sc = rows[u] > 0 ? t.gamma[ch[u]] * rsqrtf(va + t.eps) : 0.f;
      float* o = t.ss + (size_t)sg[u] * 2 * t.C;
      o[ch[u]] = sc;
      o[t.C + ch[u]] = rows[u] > 0 ? t.beta[ch[u]] - mu * sc : 0.f;
    }
  }
  if (lane == leader) atomicExch(t.ticket, 0);
}

// BN scale / shift computed by the CONSUMING conv from the producer's epilogue
// sums (the h3 direct kernel's input BN on load, X6DStats.aff_*): every block
// writes the rows of all nseg videos into `ss` (identical values from every
// block), drains its stores and then DMAs them as it does a finalize's rows --
// the finalize dispatch is gone and its latency overlaps the consumer's start.
// Armed by the host around the consumer's launches (rnb_bn_aff_arm); a launch
// whose in_ss is the armed `ss` computes them. The armed state (like the BN
// tail's) is process-global: the host thread that arms it launches the conv
// (runner lanes launch from the runner's one thread).
struct BnAffSums {
  const double* sums;        // [nseg][2][sums_c]
  int sums_c, nseg, rpc;
  const int* coffs;          // [nseg + 1] clip offsets
  const float* gamma;
  const float* beta;
  float eps;
  float* ss;                 // [nseg][2][C] out (C = the consumer's Cin_p)
};
// host: the armed descriptor, or null; a launch that uses it marks it (defined
// in bn_ops.hip)
const BnAffSums* bn_aff_armed();
void bn_aff_mark_used();
