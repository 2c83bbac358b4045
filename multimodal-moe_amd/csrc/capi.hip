// Error plumbing, identification and the launch profiler of the C-ABI
// (include/moe_hip.h).
#include <vector>

#include "moe_common.h"
#include "prof.h"

namespace moe {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const std::string& msg) {
  set_error(msg);
  return -1;
}

int check_launch(const char* what) {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(err));
    return -(1000 + (int)err);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// launch profiler: while enabled, every kernel launch of the library carries a
// hipEvent pair stamped by its dispatch (not thread-safe; profiling only)
// ---------------------------------------------------------------------------
namespace {
struct Record {
  int kind;
  hipEvent_t start, stop;
  double bytes_fixed, bytes_per_row, flops_per_row;
  int rows_slot;  // index into the pinned rows buffer, or -1
};
struct Profiler {
  bool on = false;
  std::vector<Record> recs;
  std::vector<hipEvent_t> pool;  // recycled events
  int32_t* rows_host = nullptr;  // pinned, one int per record that reads device rows
  int rows_cap = 0, rows_used = 0;

  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void clear() {
    for (auto& r : recs) {
      pool.push_back(r.start);
      pool.push_back(r.stop);
    }
    recs.clear();
    rows_used = 0;
  }
};
Profiler g_prof;
}  // namespace

ProfScope::ProfScope(hipStream_t s, int kind, double bytes_fixed, const int32_t* dev_rows, double bytes_per_row,
                     double flops_per_row)
    : stream_(s), active_(g_prof.on), idx_(-1) {
  if (!active_) return;
  Record r{kind, g_prof.ev(), g_prof.ev(), bytes_fixed, bytes_per_row, flops_per_row, -1};
  if (dev_rows != nullptr) {
    if (g_prof.rows_used >= g_prof.rows_cap) {
      const int cap = g_prof.rows_cap ? 2 * g_prof.rows_cap : 4096;
      int32_t* nb = nullptr;
      if (hipHostMalloc(reinterpret_cast<void**>(&nb), cap * sizeof(int32_t)) == hipSuccess) {
        if (g_prof.rows_host) {
          (void)hipDeviceSynchronize();
          std::copy(g_prof.rows_host, g_prof.rows_host + g_prof.rows_used, nb);
          (void)hipHostFree(g_prof.rows_host);
        }
        g_prof.rows_host = nb;
        g_prof.rows_cap = cap;
      }
    }
    if (g_prof.rows_used < g_prof.rows_cap) {
      r.rows_slot = g_prof.rows_used++;
      dev_rows_ = dev_rows;
    }
  }
  g_prof.recs.push_back(r);
  idx_ = (int)g_prof.recs.size() - 1;
}

hipEvent_t ProfScope::start_event() const { return g_prof.recs[idx_].start; }
hipEvent_t ProfScope::stop_event() const { return g_prof.recs[idx_].stop; }

ProfScope::~ProfScope() {
  if (!active_ || idx_ < 0) return;
  Record& r = g_prof.recs[idx_];
  if (r.rows_slot >= 0)  // stream-ordered read of the device row count (after the kernel)
    (void)hipMemcpyAsync(g_prof.rows_host + r.rows_slot, dev_rows_, sizeof(int32_t), hipMemcpyDeviceToHost,
                         stream_);
}

}  // namespace moe

extern "C" const char* moe_last_error(void) { return moe::g_last_error.c_str(); }

extern "C" const char* moe_version(void) { return "moe_hip 0.2.0 gfx950"; }

extern "C" int moe_profile_enable(int on) {
  moe::g_prof.clear();
  moe::g_prof.on = on != 0;
  return 0;
}

extern "C" int moe_profile_count(void) { return (int)moe::g_prof.recs.size(); }

extern "C" int moe_profile_get(int i, int* kind, float* ms, double* flops, double* bytes) {
  if (i < 0 || i >= (int)moe::g_prof.recs.size()) return moe::fail("moe_profile_get: index out of range");
  auto& r = moe::g_prof.recs[i];
  if (hipEventSynchronize(r.stop) != hipSuccess) return moe::fail("moe_profile_get: event sync failed");
  if (r.rows_slot >= 0) (void)hipDeviceSynchronize();  // the rows copy trails the stop event
  float t = 0.f;
  const hipError_t e = hipEventElapsedTime(&t, r.start, r.stop);
  if (e != hipSuccess) return moe::fail(std::string("moe_profile_get: ") + hipGetErrorString(e));
  *kind = r.kind;
  *ms = t;
  const double rows = r.rows_slot >= 0 ? (double)moe::g_prof.rows_host[r.rows_slot] : 0.0;
  *flops = r.flops_per_row * rows;
  *bytes = r.bytes_fixed + r.bytes_per_row * rows;
  return 0;
}

extern "C" int moe_profile_clear(void) {
  moe::g_prof.clear();
  return 0;
}
