// Dynamic-LDS opt-in for kernels that use more than the default 64 KB.
//
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is a per-device property of
// a kernel, so the "already set" memo is keyed by (kernel, device). A
// process-wide bool per kernel would leave the limit unset on the second
// device a process launches on. Runner replicas launch from several threads,
// hence the mutex (one uncontended lock per launch).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

static inline void rnb_ensure_max_lds(const void* kernel, int bytes = 160 * 1024) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert(std::make_pair(kernel, dev)).second)
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
