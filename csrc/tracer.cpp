// Kernel-activity tracer on rocprofiler-sdk: the MI355X equivalent of the
// reference's CUPTI bridge (reference: utils/cupti.cpp:1-175).
//
// Same contract as the reference module (initialize / flush / report of
// (kernel name, start ns, end ns), report clears), exposed as a C ABI for
// ctypes. rnb_tracer_initialize() registers this library as a
// rocprofiler-sdk tool with rocprofiler_force_configure(); the tool
//   * records kernel names from the code-object callback service
//     (DEVICE_KERNEL_SYMBOL_REGISTER: kernel_id -> name), and
//   * collects KERNEL_DISPATCH records through a lossless buffer whose
//     callback appends (kernel_id, start, end, agent) to an in-memory vector.
// rnb_tracer_flush() drains the buffer. Like every rocprofiler-sdk tool it must
// be configured before the HIP/HSA runtime initialises (i.e. before the first
// torch.cuda call in the process).
#include <rocprofiler-sdk/buffer.h>
#include <rocprofiler-sdk/buffer_tracing.h>
#include <rocprofiler-sdk/callback_tracing.h>
#include <rocprofiler-sdk/context.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct Record {
  uint64_t kernel_id;
  uint64_t begin_ns;
  uint64_t end_ns;
  uint64_t agent;
};

std::mutex g_mu;
std::vector<Record> g_records;
std::unordered_map<uint64_t, std::string> g_names;
rocprofiler_context_id_t g_ctx{};
rocprofiler_buffer_id_t g_buf{};
bool g_configured = false;
bool g_started = false;
int g_status = 0;

void code_object_cb(rocprofiler_callback_tracing_record_t record, rocprofiler_user_data_t*,
                    void*) {
  if (record.kind != ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT) return;
  if (record.operation != ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER) return;
  if (record.phase != ROCPROFILER_CALLBACK_PHASE_LOAD) return;
  auto* data =
      static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(
          record.payload);
  std::lock_guard<std::mutex> guard(g_mu);
  g_names[data->kernel_id] = data->kernel_name ? data->kernel_name : "<kernel>";
}

void buffer_cb(rocprofiler_context_id_t, rocprofiler_buffer_id_t,
               rocprofiler_record_header_t** headers, size_t num_headers, void*, uint64_t) {
  std::lock_guard<std::mutex> guard(g_mu);
  for (size_t i = 0; i < num_headers; ++i) {
    const rocprofiler_record_header_t* h = headers[i];
    if (h->category != ROCPROFILER_BUFFER_CATEGORY_TRACING ||
        h->kind != ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH)
      continue;
    auto* rec = static_cast<const rocprofiler_buffer_tracing_kernel_dispatch_record_t*>(
        h->payload);
    g_records.push_back(Record{rec->dispatch_info.kernel_id, rec->start_timestamp,
                               rec->end_timestamp, rec->dispatch_info.agent_id.handle});
  }
}

#define CHECK_RP(call, code)                             \
  do {                                                   \
    if ((call) != ROCPROFILER_STATUS_SUCCESS) {          \
      g_status = (code);                                 \
      return -1;                                         \
    }                                                    \
  } while (0)

int tool_init(rocprofiler_client_finalize_t, void*) {
  CHECK_RP(rocprofiler_create_context(&g_ctx), -10);
  CHECK_RP(rocprofiler_configure_callback_tracing_service(
               g_ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT, nullptr, 0, code_object_cb,
               nullptr),
           -11);
  const size_t buf_bytes = 4u << 20;
  CHECK_RP(rocprofiler_create_buffer(g_ctx, buf_bytes, buf_bytes - (buf_bytes >> 3),
                                     ROCPROFILER_BUFFER_POLICY_LOSSLESS, buffer_cb, nullptr,
                                     &g_buf),
           -12);
  CHECK_RP(rocprofiler_configure_buffer_tracing_service(
               g_ctx, ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH, nullptr, 0, g_buf),
           -13);
  CHECK_RP(rocprofiler_start_context(g_ctx), -14);
  g_started = true;
  return 0;
}

void tool_fini(void*) {
  if (g_started) {
    rocprofiler_flush_buffer(g_buf);
    rocprofiler_stop_context(g_ctx);
    g_started = false;
  }
}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t,
                                               rocprofiler_client_id_t* id) {
  id->name = "rnb_amd.tracer";
  static rocprofiler_tool_configure_result_t cfg = {
      sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini, nullptr};
  return &cfg;
}

}  // namespace

extern "C" {

int rnb_tracer_status() { return g_status; }

int rnb_tracer_initialize(size_t /*buffer_bytes*/) {
  if (g_configured) return 0;
  if (rocprofiler_force_configure(&configure) != ROCPROFILER_STATUS_SUCCESS) return -1;
  g_configured = true;
  return 0;
}

int rnb_tracer_started() { return g_started ? 1 : 0; }

int rnb_tracer_flush() {
  if (!g_started) return -1;
  return rocprofiler_flush_buffer(g_buf) == ROCPROFILER_STATUS_SUCCESS ? 0 : -2;
}

int rnb_tracer_count() {
  std::lock_guard<std::mutex> guard(g_mu);
  return (int)g_records.size();
}

// Copies record i; name truncated to name_cap-1 bytes. Returns the full name length.
int rnb_tracer_fetch(int i, char* name, int name_cap, uint64_t* begin_ns, uint64_t* end_ns,
                     int* op, int* device) {
  std::lock_guard<std::mutex> guard(g_mu);
  if (i < 0 || i >= (int)g_records.size()) return -1;
  const Record& r = g_records[i];
  auto it = g_names.find(r.kernel_id);
  const std::string nm = it != g_names.end() ? it->second : std::string("<kernel>");
  if (name && name_cap > 0) {
    const int n = (int)nm.size() < name_cap - 1 ? (int)nm.size() : name_cap - 1;
    std::memcpy(name, nm.data(), n);
    name[n] = '\0';
  }
  *begin_ns = r.begin_ns;
  *end_ns = r.end_ns;
  *op = 0;
  *device = (int)r.agent;
  return (int)nm.size();
}

void rnb_tracer_clear() {
  std::lock_guard<std::mutex> guard(g_mu);
  g_records.clear();
}

int rnb_tracer_finalize() {
  tool_fini(nullptr);
  return 0;
}

const char* rnb_tracer_error() { return "see rnb_tracer_status()"; }

}  // extern "C"
