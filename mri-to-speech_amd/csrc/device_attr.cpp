// Per-device launch attributes for libm2s launchers (m2s_common.hpp).  Function-local statics in the
// launchers would fix these at the first device that called them; engines on several devices in one
// process need them per device.
#include <map>
#include <mutex>
#include <utility>

#include "m2s_common.hpp"

namespace m2s {

namespace {
std::mutex g_mu;
int cur_device() {
  int d = 0;
  M2S_HIP(hipGetDevice(&d));
  return d;
}
}  // namespace

int device_cus() {
  static std::map<int, int> cache;
  const int d = cur_device();
  std::lock_guard<std::mutex> l(g_mu);
  auto it = cache.find(d);
  if (it != cache.end()) return it->second;
  int v = 0;
  M2S_HIP(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d));
  return cache[d] = v > 0 ? v : 256;
}

void allow_lds(const void* kernel) {
  static std::map<std::pair<int, const void*>, bool> done;
  const int d = cur_device();
  std::lock_guard<std::mutex> l(g_mu);
  bool& f = done[{d, kernel}];
  if (!f) {
    M2S_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    f = true;
  }
}

int device_resident(const void* kernel, int block, size_t lds) {
  const int cus = device_cus();
  static std::map<std::pair<int, const void*>, int> cache;
  const int d = cur_device();
  std::lock_guard<std::mutex> l(g_mu);
  auto it = cache.find({d, kernel});
  if (it != cache.end()) return it->second;
  int per_cu = 0;
  M2S_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds));
  return cache[{d, kernel}] = cus * per_cu;
}

}  // namespace m2s
