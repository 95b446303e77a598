// Event-based per-kernel timing used by bench.py's roofline figure (m2s_prof_* in m2s.h).
#pragma once

#include <string>

#include "m2s_common.hpp"

namespace m2s {

bool prof_on();
// Brackets one kernel launch with HIP events on `s` when profiling is enabled.
// Stage label (e.g. "cnn", "bilstm", "mrf_c128") of the launches recorded while a StageTag lives on this
// thread; nested tags restore the outer one.  bench.py's roofline.stages and tools/evidence.py's per-stage PMC
// records group launches by it (m2s_prof_launches).
class StageTag {
 public:
  explicit StageTag(const std::string& stage);
  ~StageTag();

 private:
  std::string prev_;
};

class ProfScope {
 public:
  // spill: bytes of an intermediate the kernel writes only for a later kernel to read back (not in `bytes`)
  ProfScope(const std::string& name, double flops, double bytes, hipStream_t s, double spill = 0.0);
  ~ProfScope();

 private:
  int slot_ = -1;
  hipStream_t s_;
};

}  // namespace m2s
