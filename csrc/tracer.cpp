// Kernel-activity tracer on roctracer: the MI355X equivalent of the
// reference's CUPTI bridge (reference: utils/cupti.cpp:1-175).
//
// Same contract as the reference Python module (initialize / flush / report
// returning (kernel name, start ns, end ns) and clearing), exposed with a C
// ABI for ctypes: rnb_tracer_initialize() opens a roctracer activity pool and
// enables HIP_OPS dispatch + copy activity; completed buffers are decoded in
// the pool callback into an in-memory vector guarded by a mutex;
// rnb_tracer_flush() forces delivery; rnb_tracer_count/fetch/clear read it.
#include <roctracer/roctracer.h>
#include <roctracer/roctracer_hip.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Record {
  std::string name;
  uint64_t begin_ns;
  uint64_t end_ns;
  uint32_t op;
  int device;
  uint64_t correlation;
};

std::mutex g_mu;
std::vector<Record> g_records;
bool g_open = false;

void buffer_callback(const char* begin, const char* end, void* /*arg*/) {
  const roctracer_record_t* rec = reinterpret_cast<const roctracer_record_t*>(begin);
  const roctracer_record_t* stop = reinterpret_cast<const roctracer_record_t*>(end);
  std::lock_guard<std::mutex> guard(g_mu);
  while (rec < stop) {
    if (rec->domain == ACTIVITY_DOMAIN_HIP_OPS) {
      Record r;
      r.begin_ns = rec->begin_ns;
      r.end_ns = rec->end_ns;
      r.op = rec->op;
      r.device = rec->device_id;
      r.correlation = rec->correlation_id;
      if (rec->op == HIP_OP_ID_DISPATCH)
        r.name = rec->kernel_name ? rec->kernel_name : "<kernel>";
      else if (rec->op == HIP_OP_ID_COPY)
        r.name = "<memcpy>";
      else
        r.name = "<barrier>";
      g_records.push_back(std::move(r));
    }
    if (roctracer_next_record(rec, &rec) != ROCTRACER_STATUS_SUCCESS) break;
  }
}

}  // namespace

extern "C" {

const char* rnb_tracer_error() { return roctracer_error_string(); }

int rnb_tracer_initialize(size_t buffer_bytes) {
  if (g_open) return 0;
  roctracer_properties_t props;
  std::memset(&props, 0, sizeof(props));
  props.buffer_size = buffer_bytes ? buffer_bytes : (size_t)(4u << 20);
  props.buffer_callback_fun = buffer_callback;
  props.buffer_callback_arg = nullptr;
  if (roctracer_open_pool(&props) != ROCTRACER_STATUS_SUCCESS) return -1;
  if (roctracer_enable_op_activity(ACTIVITY_DOMAIN_HIP_OPS, HIP_OP_ID_DISPATCH) !=
      ROCTRACER_STATUS_SUCCESS)
    return -2;
  if (roctracer_enable_op_activity(ACTIVITY_DOMAIN_HIP_OPS, HIP_OP_ID_COPY) !=
      ROCTRACER_STATUS_SUCCESS)
    return -3;
  g_open = true;
  return 0;
}

int rnb_tracer_flush() {
  if (!g_open) return -1;
  return roctracer_flush_activity() == ROCTRACER_STATUS_SUCCESS ? 0 : -2;
}

int rnb_tracer_count() {
  std::lock_guard<std::mutex> guard(g_mu);
  return (int)g_records.size();
}

// Copies record i; name truncated to name_cap-1 bytes. Returns full name length.
int rnb_tracer_fetch(int i, char* name, int name_cap, uint64_t* begin_ns, uint64_t* end_ns,
                     int* op, int* device) {
  std::lock_guard<std::mutex> guard(g_mu);
  if (i < 0 || i >= (int)g_records.size()) return -1;
  const Record& r = g_records[i];
  if (name && name_cap > 0) {
    const int n = (int)r.name.size() < name_cap - 1 ? (int)r.name.size() : name_cap - 1;
    std::memcpy(name, r.name.data(), n);
    name[n] = '\0';
  }
  *begin_ns = r.begin_ns;
  *end_ns = r.end_ns;
  *op = (int)r.op;
  *device = r.device;
  return (int)r.name.size();
}

void rnb_tracer_clear() {
  std::lock_guard<std::mutex> guard(g_mu);
  g_records.clear();
}

int rnb_tracer_finalize() {
  if (!g_open) return 0;
  roctracer_disable_op_activity(ACTIVITY_DOMAIN_HIP_OPS, HIP_OP_ID_DISPATCH);
  roctracer_disable_op_activity(ACTIVITY_DOMAIN_HIP_OPS, HIP_OP_ID_COPY);
  roctracer_flush_activity();
  roctracer_close_pool();
  g_open = false;
  return 0;
}

}  // extern "C"
