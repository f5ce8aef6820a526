// Native runtime services for the rnb_amd engine (host code, HIP runtime API).
//
//  * HIP IPC export/import of producer-owned slot buffers and events -- the
//    MI355X replacement for the reference's CUDA-IPC shared TensorEvents
//    (reference: control.py:19-46, 151-157).
//  * async / peer copies (hipMemcpyAsync with hipMemcpyDefault routes a
//    cross-GPU copy over xGMI through the SDMA engines).
//  * a small device allocator wrapper so slot memory is a dedicated
//    allocation (IPC handles then map exactly one slot).
//
// Exposed with a C ABI and loaded through ctypes (rnb_amd/ops/native.py).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstring>
#include <cstdint>

extern "C" {

const char* rnb_error_string(int err) { return hipGetErrorString((hipError_t)err); }

int rnb_set_device(int dev) { return (int)hipSetDevice(dev); }

int rnb_get_device(int* dev) { return (int)hipGetDevice(dev); }

int rnb_device_count(int* n) { return (int)hipGetDeviceCount(n); }

int rnb_malloc(void** ptr, size_t bytes) { return (int)hipMalloc(ptr, bytes); }

int rnb_free(void* ptr) { return (int)hipFree(ptr); }

// host-coherent, device-mapped memory (a flag the GPU writes and the host
// reads after the work completes, with no copy): *host and *dev address it
int rnb_host_alloc_mapped(size_t bytes, void** host, void** dev) {
  hipError_t e = hipHostMalloc(host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  std::memset(*host, 0, bytes);
  return (int)hipHostGetDevicePointer(dev, *host, 0);
}

int rnb_host_free(void* host) { return (int)hipHostFree(host); }

int rnb_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

int rnb_ipc_get_mem_handle(void* ptr, void* out_handle) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return (int)e;
  std::memcpy(out_handle, &h, sizeof(h));
  return 0;
}

int rnb_ipc_open_mem_handle(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int rnb_ipc_close_mem_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// interprocess events: created with hipEventInterprocess | hipEventDisableTiming
int rnb_ipc_event_create(void** ev) {
  hipEvent_t e;
  hipError_t r = hipEventCreateWithFlags(&e, hipEventInterprocess | hipEventDisableTiming);
  *ev = (void*)e;
  return (int)r;
}

int rnb_ipc_event_handle_size() { return (int)sizeof(hipIpcEventHandle_t); }

int rnb_ipc_get_event_handle(void* ev, void* out_handle) {
  hipIpcEventHandle_t h;
  hipError_t e = hipIpcGetEventHandle(&h, (hipEvent_t)ev);
  if (e != hipSuccess) return (int)e;
  std::memcpy(out_handle, &h, sizeof(h));
  return 0;
}

int rnb_ipc_open_event_handle(const void* handle, void** ev) {
  hipIpcEventHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  hipEvent_t e;
  hipError_t r = hipIpcOpenEventHandle(&e, h);
  *ev = (void*)e;
  return (int)r;
}

int rnb_event_record(void* ev, void* stream) {
  return (int)hipEventRecord((hipEvent_t)ev, (hipStream_t)stream);
}

int rnb_stream_wait_event(void* stream, void* ev) {
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0);
}

int rnb_event_synchronize(void* ev) { return (int)hipEventSynchronize((hipEvent_t)ev); }

int rnb_event_query(void* ev) { return (int)hipEventQuery((hipEvent_t)ev); }

// returns and clears the thread's last HIP error (a tolerated failure must not
// surface later through a kernel wrapper's hipGetLastError)
int rnb_clear_last_error() { return (int)hipGetLastError(); }

int rnb_event_destroy(void* ev) { return (int)hipEventDestroy((hipEvent_t)ev); }

int rnb_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream);
}

int rnb_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  return (int)hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
}

int rnb_memcpy_peer_async(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes,
                          void* stream) {
  return (int)hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, (hipStream_t)stream);
}

int rnb_stream_synchronize(void* stream) { return (int)hipStreamSynchronize((hipStream_t)stream); }

// raw HIP streams (scripts/ipc_event_matrix.py compares them with torch's)
int rnb_stream_create(int nonblocking, int priority, void** stream) {
  hipStream_t s;
  const hipError_t e = hipStreamCreateWithPriority(&s, nonblocking ? hipStreamNonBlocking : 0,
                                                   priority);
  *stream = (void*)s;
  return (int)e;
}

int rnb_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

// a stream whose dispatches may only use the CUs whose bits are set in
// ``mask`` (n_words 32-bit words, CU i = bit i % 32 of word i / 32): a replica
// group kept off part of the chip so that another group's calls find those
// CUs free (bench.py --small-cu-frac)
int rnb_stream_create_cumask(const uint32_t* mask, int n_words, void** stream) {
  hipStream_t s;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask);
  *stream = (void*)s;
  return (int)e;
}

// ~cycles of busy wait on the stream (a pending record for the IPC-event tests)
__global__ void rnb_spin_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

int rnb_spin(void* stream, long long cycles) {
  hipLaunchKernelGGL(rnb_spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, cycles);
  return (int)hipGetLastError();
}

int rnb_can_access_peer(int dev, int peer, int* out) {
  return (int)hipDeviceCanAccessPeer(out, dev, peer);
}

int rnb_mem_get_info(size_t* free_b, size_t* total_b) { return (int)hipMemGetInfo(free_b, total_b); }

}  // extern "C"
