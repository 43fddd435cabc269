/*!
 * \file speed_test.cc
 * \brief Collective speed test (the shape of the reference's test/speed_test.cc): nrep rounds
 *        of Allreduce<Max>, Allreduce<Sum> (float32 x n) and Broadcast (n bytes from a
 *        random root); prints per-op mean/std time across ranks and rabit's MB/s speed line
 *        (per-rank algorithm bandwidth), plus nccl-tests style busbw.
 *        device=1 puts the buffers in HBM (hipMalloc) so the RCCL/xGMI plane is measured.
 * Usage: speed_test <ndata> <nrepeat> [device=1] [rabit params...]
 */
#include <hip/hip_runtime_api.h>
#include <rabit/internal/timer.h>
#include <rabit/rabit.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace {
double g_max, g_sum, g_bcast;

void Report(const char *name, double t, size_t n, int nrep, size_t elem, bool allreduce) {
  const int world = rabit::GetWorldSize();
  double tsum = t;
  rabit::Allreduce<rabit::op::Sum>(&tsum, 1);
  const double mean = tsum / world;
  double dev2 = (t - mean) * (t - mean);
  rabit::Allreduce<rabit::op::Sum>(&dev2, 1);
  if (rabit::GetRank() != 0) return;
  rabit::TrackerPrintf("%s: mean=%g, std=%g sec\n", name, mean, std::sqrt(dev2 / world));
  if (n != 0) {
    const double bytes = static_cast<double>(n) * nrep * elem;
    const double algbw = bytes / mean;
    const double busbw = allreduce && world > 1 ? algbw * 2.0 * (world - 1) / world : algbw;
    rabit::TrackerPrintf("%s-speed: %g MB/sec (algbw %.2f GB/s, busbw %.2f GB/s)\n", name,
                         algbw / 1024 / 1024, algbw / 1e9, busbw / 1e9);
  }
}
}  // namespace

int main(int argc, char *argv[]) {
  if (argc < 3) {
    printf("Usage: speed_test <ndata> <nrepeat> [device=1]\n");
    return 0;
  }
  const size_t n = static_cast<size_t>(atol(argv[1]));
  const int nrep = atoi(argv[2]);
  bool on_device = false;
  for (int i = 3; i < argc; ++i) {
    if (!strcmp(argv[i], "device=1")) on_device = true;
  }
  rabit::utils::Check(nrep >= 1, "need at least one repetition");
  rabit::Init(argc, argv);
  const int rank = rabit::GetRank();
  const int world = rabit::GetWorldSize();
  // broadcast roots from a generator of our own: the reference draws them with rand(), whose
  // global state the GPU runtime may advance by different amounts on different ranks (seen with
  // HBM staging: ranks disagreed on the root and the job desynchronised)
  std::mt19937 roots(0);
  std::vector<float> host(n);
  std::string bstr(n, '\0');
  float *fbuf = host.data();
  char *bbuf = &bstr[0];
  if (on_device) {
    rabit::utils::Check(hipMalloc(reinterpret_cast<void **>(&fbuf), n * sizeof(float)) ==
                                hipSuccess &&
                            hipMalloc(reinterpret_cast<void **>(&bbuf), n) == hipSuccess,
                        "hipMalloc failed");
  }
  const double t0 = rabit::utils::GetTime();
  for (int rep = 0; rep < nrep; ++rep) {
    for (size_t i = 0; i < n; ++i) host[i] = static_cast<float>((i * (rank + 1)) % 111);
    if (on_device) (void)hipMemcpy(fbuf, host.data(), n * sizeof(float), hipMemcpyHostToDevice);
    double t = rabit::utils::GetTime();
    rabit::Allreduce<rabit::op::Max>(fbuf, n);
    if (on_device) (void)hipDeviceSynchronize();
    g_max += rabit::utils::GetTime() - t;

    for (size_t i = 0; i < n; ++i) host[i] = static_cast<float>((i * (rank + 1)) % 131);
    if (on_device) (void)hipMemcpy(fbuf, host.data(), n * sizeof(float), hipMemcpyHostToDevice);
    t = rabit::utils::GetTime();
    rabit::Allreduce<rabit::op::Sum>(fbuf, n);
    if (on_device) (void)hipDeviceSynchronize();
    g_sum += rabit::utils::GetTime() - t;

    const int root = static_cast<int>(roots() % static_cast<unsigned>(world));
    t = rabit::utils::GetTime();
    rabit::Broadcast(bbuf, n, root);
    if (on_device) (void)hipDeviceSynchronize();
    g_bcast += rabit::utils::GetTime() - t;
  }
  const double tot = rabit::utils::GetTime() - t0;
  Report("max_tdiff", g_max, n, nrep, sizeof(float), true);
  Report("sum_tdiff", g_sum, n, nrep, sizeof(float), true);
  Report("bcast_tdiff", g_bcast, n, nrep, sizeof(char), false);
  Report("tot_tdiff", tot, 0, nrep, sizeof(float), false);
  if (on_device) {
    (void)hipFree(fbuf);
    (void)hipFree(bbuf);
  }
  rabit::Finalize();
  return 0;
}
