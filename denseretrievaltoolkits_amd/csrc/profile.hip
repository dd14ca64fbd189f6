// Launch-timing hooks: hipEvent pairs recorded on the launch stream.
#include "profile.h"

#include <mutex>
#include <vector>

#include "drt_common.h"

namespace drt {

namespace {
std::mutex g_mu;
bool g_on[PROF_N] = {false, false, false, false, false};
std::vector<ProfPair> g_rec[PROF_N];
std::vector<hipEvent_t> g_pool;

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

ProfPair prof_begin(int family, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (family < 0 || family >= PROF_N || !g_on[family]) return {nullptr, nullptr};
  ProfPair p{take_event(), take_event()};
  if (!p.a || !p.b) return {nullptr, nullptr};
  if (hipEventRecord(p.a, s) != hipSuccess) return {nullptr, nullptr};
  g_rec[family].push_back(p);
  return p;
}

void prof_end(const ProfPair& p, hipStream_t s) {
  if (p.b) (void)hipEventRecord(p.b, s);
}

}  // namespace drt

using namespace drt;

extern "C" int drt_profile_enable(int32_t family, int32_t enable) {
  if (family < 0 || family >= PROF_N) return DRT_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  g_on[family] = enable != 0;
  return DRT_OK;
}

extern "C" int drt_profile_read_each(int32_t family, double* ms_each, int64_t cap, int64_t* count) {
  if (family < 0 || family >= PROF_N || cap < 0 || (cap > 0 && !ms_each)) return DRT_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  int64_t n = 0;
  for (auto& p : g_rec[family]) {
    hipError_t e = hipEventSynchronize(p.b);
    if (e != hipSuccess) return (int)e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, p.a, p.b);
    if (e != hipSuccess) return (int)e;
    if (n < cap) ms_each[n] = ms;
    ++n;
    g_pool.push_back(p.a);
    g_pool.push_back(p.b);
  }
  g_rec[family].clear();
  if (count) *count = n;
  return DRT_OK;
}

extern "C" int drt_profile_read(int32_t family, double* total_ms, int64_t* count) {
  if (family < 0 || family >= PROF_N) return DRT_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  double tot = 0.0;
  int64_t n = 0;
  for (auto& p : g_rec[family]) {
    hipError_t e = hipEventSynchronize(p.b);
    if (e != hipSuccess) return (int)e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, p.a, p.b);
    if (e != hipSuccess) return (int)e;
    tot += ms;
    ++n;
    g_pool.push_back(p.a);
    g_pool.push_back(p.b);
  }
  g_rec[family].clear();
  if (total_ms) *total_ms = tot;
  if (count) *count = n;
  return DRT_OK;
}
