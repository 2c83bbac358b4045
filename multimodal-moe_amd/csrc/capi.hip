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
  int rows_slot;  // index into the device rows buffer, or -1
  bool per_row;   // false: flops_per_row is the launch's total flops
};
constexpr int kRowSlots = 1 << 16;
struct Profiler {
  bool on = false;
  std::vector<Record> recs;
  std::vector<hipEvent_t> pool;   // free events (created at enable, recycled at clear)
  int32_t* rows_dev = nullptr;    // kRowSlots device ints the kernels write their row counts to
  std::vector<int32_t> rows_host;
  int rows_used = 0;
  bool rows_fetched = false;

  void reserve(int n) {
    while ((int)pool.size() < n) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) break;
      pool.push_back(e);
    }
  }
  hipEvent_t ev() {
    if (pool.empty()) reserve(256);
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  void clear() {
    for (auto& r : recs) {
      pool.push_back(r.start);
      pool.push_back(r.stop);
    }
    recs.clear();
    rows_used = 0;
    rows_fetched = false;
  }
};
Profiler g_prof;
// host-side launch counts per profiler kind: every launch through a ProfScope,
// profiling on or off and inside hipGraph capture (a captured launch counts
// once, at capture) -- how a caller checks that the HIP path ran
constexpr int kKinds = 32;
long long g_launches[kKinds] = {};
}  // namespace

ProfScope::ProfScope(hipStream_t s, int kind, double bytes_fixed, bool per_row, double bytes_per_row,
                     double flops_per_row)
    : active_(g_prof.on), idx_(-1) {
  (void)s;
  if (kind >= 0 && kind < kKinds) ++g_launches[kind];
  if (!active_) return;
  Record r{kind, g_prof.ev(), g_prof.ev(), bytes_fixed, bytes_per_row, flops_per_row, -1, per_row};
  if (per_row && g_prof.rows_dev != nullptr && g_prof.rows_used < kRowSlots) r.rows_slot = g_prof.rows_used++;
  g_prof.recs.push_back(r);
  idx_ = (int)g_prof.recs.size() - 1;
}

hipEvent_t ProfScope::start_event() const { return g_prof.recs[idx_].start; }
hipEvent_t ProfScope::stop_event() const { return g_prof.recs[idx_].stop; }
int32_t* ProfScope::rows_slot() const {
  if (!active()) return nullptr;
  const int slot = g_prof.recs[idx_].rows_slot;
  return slot >= 0 ? g_prof.rows_dev + slot : nullptr;
}

}  // namespace moe

extern "C" const char* moe_last_error(void) { return moe::g_last_error.c_str(); }

extern "C" const char* moe_version(void) { return "moe_hip 0.2.0 gfx950"; }

extern "C" int moe_profile_enable(int on) {
  auto& P = moe::g_prof;
  P.clear();
  P.on = on != 0;
  if (P.on) {
    P.reserve(8192);  // no event creation inside a profiled region of up to 4096 launches
    if (P.rows_dev == nullptr &&
        hipMalloc(reinterpret_cast<void**>(&P.rows_dev), moe::kRowSlots * sizeof(int32_t)) != hipSuccess) {
      P.rows_dev = nullptr;
      return moe::fail("moe_profile_enable: cannot allocate the row-count slots");
    }
  }
  return 0;
}

extern "C" int moe_profile_count(void) { return (int)moe::g_prof.recs.size(); }

extern "C" int moe_profile_get(int i, int* kind, float* ms, double* flops, double* bytes) {
  if (i < 0 || i >= (int)moe::g_prof.recs.size()) return moe::fail("moe_profile_get: index out of range");
  auto& P = moe::g_prof;
  auto& r = P.recs[i];
  if (hipEventSynchronize(r.stop) != hipSuccess) return moe::fail("moe_profile_get: event sync failed");
  if (r.rows_slot >= 0 && !P.rows_fetched) {  // one copy of every slot written so far
    P.rows_host.resize(P.rows_used);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(P.rows_host.data(), P.rows_dev, P.rows_used * sizeof(int32_t), hipMemcpyDeviceToHost) !=
            hipSuccess)
      return moe::fail("moe_profile_get: row-count copy failed");
    P.rows_fetched = true;
  }
  float t = 0.f;
  const hipError_t e = hipEventElapsedTime(&t, r.start, r.stop);
  if (e != hipSuccess) return moe::fail(std::string("moe_profile_get: ") + hipGetErrorString(e));
  *kind = r.kind;
  *ms = t;
  const double rows = r.rows_slot >= 0 ? (double)P.rows_host[r.rows_slot] : 0.0;
  *flops = r.per_row ? r.flops_per_row * rows : r.flops_per_row;
  *bytes = r.bytes_fixed + r.bytes_per_row * rows;
  return 0;
}

extern "C" int moe_profile_clear(void) {
  moe::g_prof.clear();
  return 0;
}

extern "C" int moe_launch_counts(long long* out, int n) {
  if (out == nullptr || n < 0) return moe::fail("moe_launch_counts: NULL out or n < 0");
  for (int i = 0; i < n; ++i) out[i] = i < moe::kKinds ? moe::g_launches[i] : 0;
  return 0;
}

extern "C" int moe_launch_counts_reset(void) {
  for (auto& c : moe::g_launches) c = 0;
  return 0;
}
