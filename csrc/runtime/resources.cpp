// Resource enforcement + tracing hooks.
//
// * CU-masked streams: the Brain's per-rank CU plan becomes a real hardware
//   restriction by creating the process's compute stream with
//   hipExtStreamCreateWithCUMask; PyTorch then runs on it as an
//   ExternalStream (easydl_amd/utils/resources.py).  Masks are given as
//   32-bit words over the 256 CUs of an MI355X.
// * roctx ranges for rocprofv3 --marker-trace, resolved with dlopen so the
//   runtime has no hard dependency on the profiler SDK (no-ops when absent).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace {
typedef int (*push_fn)(const char*);
typedef int (*pop_fn)();
typedef void (*mark_fn)(const char*);
push_fn g_push = nullptr;
pop_fn g_pop = nullptr;
mark_fn g_mark = nullptr;
bool g_tried = false;

void load_roctx() {
  if (g_tried) return;
  g_tried = true;
  const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                         "libroctx64.so"};
  for (const char* n : names) {
    void* h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
    if (!h) continue;
    g_push = (push_fn)dlsym(h, "roctxRangePushA");
    g_pop = (pop_fn)dlsym(h, "roctxRangePop");
    g_mark = (mark_fn)dlsym(h, "roctxMarkA");
    if (g_push && g_pop) return;
  }
}
}  // namespace

extern "C" {

// Returns a hipStream_t (as void*) restricted to the CUs set in mask, or null.
void* edl_stream_create_cumask(int device, const uint32_t* mask, int nwords, int priority) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return nullptr;
  (void)priority;
  return s;
}

int edl_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

// The CU mask a stream's kernels are restricted to (32-bit words over the CUs);
// returns a hipError_t.  Lets tests check every stream of a CU-planned rank.
int edl_stream_get_cumask(void* s, uint32_t* out, int nwords) {
  return (int)hipExtStreamGetCUMask((hipStream_t)s, (uint32_t)nwords, out);
}

int edl_roctx_available() {
  load_roctx();
  return g_push != nullptr;
}
int edl_roctx_push(const char* msg) {
  load_roctx();
  return g_push ? g_push(msg) : -1;
}
int edl_roctx_pop() {
  load_roctx();
  return g_pop ? g_pop() : -1;
}
void edl_roctx_mark(const char* msg) {
  load_roctx();
  if (g_mark) g_mark(msg);
}

}  // extern "C"
