// nconv_occ.hip — the device properties launchers size their grids by (CU count, resident
// workgroups of a kernel), cached per device ordinal behind a mutex: several host threads may
// drive several devices at once (one replica per device), and a host may mix GPU models.
#include <map>
#include <mutex>
#include <utility>

#include "nconv_internal.h"

namespace nconv {

namespace {
std::mutex g_occ_mu;
std::map<int, int> g_cus;                                  // device -> CUs
std::map<std::pair<int, const void*>, int> g_per_cu;       // (device, kernel) -> workgroups per CU
int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return dev;
}
}  // namespace

int dev_cus() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_cus.find(dev);
    if (it != g_cus.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_cus[dev] = n;
    return n;
}

int dev_occupancy(const void* kernel, int threads, size_t dyn_lds) {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    const auto key = std::make_pair(dev, kernel);
    auto it = g_per_cu.find(key);
    if (it != g_per_cu.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, dyn_lds) != hipSuccess || n <= 0) n = 1;
    g_per_cu[key] = n;  // (a kernel's dynamic LDS is fixed per instantiation here)
    return n;
}

}  // namespace nconv
