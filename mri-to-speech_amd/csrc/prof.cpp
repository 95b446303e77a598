#include "prof.hpp"

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/m2s.h"

namespace m2s {
namespace {

thread_local std::string g_stage = "other";

struct Rec {
  std::string name, stage;
  double flops, bytes, spill;
  hipEvent_t a, b;
};

struct Prof {
  std::mutex mu;
  bool on = false;
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    // timing-only events: no system-scope fence when recorded (no cache write-back / invalidate around the
    // launches they bracket; the durations agree with rocprofv3's trace of the same steps either way,
    // tools/step_kstats.py)
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) M2S_HIP(hipEventCreate(&e));
    return e;
  }
};

Prof& P() {
  static Prof p;
  return p;
}

}  // namespace

bool prof_on() { return P().on; }

StageTag::StageTag(const std::string& stage) : prev_(g_stage) { g_stage = stage; }
StageTag::~StageTag() { g_stage = prev_; }

ProfScope::ProfScope(const std::string& name, double flops, double bytes, hipStream_t s, double spill) : s_(s) {
  Prof& p = P();
  if (!p.on) return;
  std::lock_guard<std::mutex> g(p.mu);
  Rec r{name, g_stage, flops, bytes, spill, p.get(), p.get()};
  M2S_HIP(hipEventRecord(r.a, s));
  slot_ = (int)p.recs.size();
  p.recs.push_back(r);
}

ProfScope::~ProfScope() {
  if (slot_ < 0) return;
  Prof& p = P();
  std::lock_guard<std::mutex> g(p.mu);
  (void)hipEventRecord(p.recs[slot_].b, s_);
}

}  // namespace m2s

using namespace m2s;

extern "C" int m2s_prof_enable_impl(int on) {
  P().on = on != 0;
  return 0;
}

extern "C" int m2s_prof_collect_impl(m2s_prof_stat* out, int max, int* n_out) {
  Prof& p = P();
  std::lock_guard<std::mutex> g(p.mu);
  std::map<std::string, m2s_prof_stat> agg;
  for (auto& r : p.recs) {
    M2S_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    M2S_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    auto& s = agg[r.name];
    std::strncpy(s.name, r.name.c_str(), sizeof(s.name) - 1);
    s.launches += 1;
    s.ms += ms;
    s.flops += r.flops;
    s.bytes += r.bytes;
    p.pool.push_back(r.a);
    p.pool.push_back(r.b);
  }
  p.recs.clear();
  int n = 0;
  for (auto& kv : agg) {
    if (n < max && out) out[n] = kv.second;
    ++n;
  }
  if (n_out) *n_out = n;
  return 0;
}

extern "C" int m2s_prof_launches_impl(m2s_prof_launch* out, int max, int* n_out) {
  Prof& p = P();
  std::lock_guard<std::mutex> g(p.mu);
  if (!out) {  // count only: the record stays
    if (n_out) *n_out = (int)p.recs.size();
    return 0;
  }
  int n = 0;
  for (auto& r : p.recs) {
    M2S_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    M2S_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    if (n < max && out) {
      m2s_prof_launch& l = out[n];
      std::memset(&l, 0, sizeof(l));
      std::strncpy(l.name, r.name.c_str(), sizeof(l.name) - 1);
      std::strncpy(l.stage, r.stage.c_str(), sizeof(l.stage) - 1);
      l.ms = ms;
      l.flops = r.flops;
      l.bytes = r.bytes;
      l.spill_bytes = r.spill;
    }
    ++n;
    p.pool.push_back(r.a);
    p.pool.push_back(r.b);
  }
  p.recs.clear();
  if (n_out) *n_out = n;
  return 0;
}
