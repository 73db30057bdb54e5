// prof.cpp — optional per-kernel-class HIP-event timing used by bench.py for the live
// roofline figure.  Events are recorded on the launch stream around each launch of a named
// kernel class; totals are read back after the caller has synchronised the stream.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace {
struct Rec {
  std::string name;
  double flops;
  hipEvent_t a, b;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;
std::vector<std::string> g_select;  // recorded classes (empty = all)

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

namespace damc_prof {
bool enabled() { return g_on; }
int begin(const char* name, double flops, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_select.empty()) {
    bool hit = false;
    for (const std::string& c : g_select) hit = hit || (name && c == name);
    if (!hit) return -1;
  }
  Rec r{name ? name : "?", flops, take_event(), take_event()};
  if (!r.a || !r.b) return -1;
  if (hipEventRecord(r.a, s) != hipSuccess) return -1;
  g_recs.push_back(r);
  return (int)g_recs.size() - 1;
}
void end(int slot, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  // a failed record leaves the slot's end event unset; damc_prof_query then returns that error
  if (slot >= 0 && slot < (int)g_recs.size()) (void)hipEventRecord(g_recs[slot].b, s);
}
}  // namespace damc_prof

extern "C" int damc_prof_enable(int on) {
  g_on = on != 0;
  return 0;
}

extern "C" int damc_prof_select(const char* classes) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_select.clear();
  if (!classes) return 0;
  std::string cur;
  for (const char* c = classes;; ++c) {
    if (*c == ',' || *c == 0) {
      if (!cur.empty()) g_select.push_back(cur);
      cur.clear();
      if (*c == 0) break;
    } else {
      cur += *c;
    }
  }
  return 0;
}

extern "C" int damc_prof_reset(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& r : g_recs) {
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
  return 0;
}

extern "C" int damc_prof_query(const char* name, double* total_ms, long* launches, double* flops) {
  if (!name || !total_ms || !launches || !flops) return DAMC_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_mu);
  double t = 0, f = 0;
  long n = 0;
  for (auto& r : g_recs) {
    if (r.name != name) continue;
    float ms = 0.f;
    hipError_t e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess) return (int)e;
    t += ms;
    f += r.flops;
    ++n;
  }
  *total_ms = t;
  *launches = n;
  *flops = f;
  return 0;
}

extern "C" int damc_abi_version(void) { return DAMC_ABI_VERSION; }

extern "C" const char* damc_error_string(int code) {
  switch (code) {
    case DAMC_OK: return "ok";
    case DAMC_ERR_ARG: return "damc: invalid argument or shape";
    case DAMC_ERR_WORKSPACE: return "damc: workspace too small";
    case DAMC_ERR_UNSUPPORTED: return "damc: unsupported configuration";
    default: return hipGetErrorString((hipError_t)code);
  }
}
