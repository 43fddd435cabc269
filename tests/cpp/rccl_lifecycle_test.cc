/*!
 * \file rccl_lifecycle_test.cc
 * \brief GPU test of the RCCL communicator lifecycle under failure (one MI355X is enough):
 *
 *  1. a 2-rank communicator whose second rank never joins: the bring-up runs on a helper
 *     thread (RCCL's init blocks in its bootstrap while a rank is missing, whatever the
 *     blocking flag says), the waiter gives up at the deadline (kTimeout) and abandons the
 *     helper, and the plane builds a working one-rank communicator afterwards;
 *  2. the same, ended early by the failure probe (a peer reported dead): kAborted well before
 *     the deadline;
 *  3. an RCCL enqueue that fails (mock_rccl_error: the call returns ncclRemoteError) becomes
 *     kAborted with the communicator dropped, not a process exit, and the next epoch works;
 *  4. three more multi-rank bring-ups that would be abandoned: the number of live abandoned
 *     helpers stays at DevicePlane::kMaxAbandonedInits (bring-ups beyond it are refused at
 *     once), a world-1 communicator still works, and the process exits cleanly.
 *
 * Exit status 0 when every check passes.  Reference: the survivor side of
 * `src/allreduce_robust.cc:687-725` (CheckAndRecover never waits forever on a dead peer).
 */
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "device/device_plane.h"
#include "device/kernels.h"

using rabit::device::DeviceConfig;
using rabit::device::DevicePlane;
using rabit::net::Status;

namespace {
int g_fail = 0;
#define CHECK_TRUE(cond, ...)                                     \
  do {                                                            \
    if (!(cond)) {                                                \
      fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      fprintf(stderr, __VA_ARGS__);                               \
      fprintf(stderr, "\n");                                      \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

/*! \brief a world-1 communicator runs a float sum correctly (the plane is usable) */
bool WorldOneWorks(DevicePlane *dev) {
  printf("    world-1 communicator...\n");
  if (dev->InitComm(DevicePlane::NewUniqueId(), 1, 0, nullptr) != Status::kSuccess) return false;
  printf("    world-1 communicator up\n");
  dev->BeginEpoch(1, 0);
  const size_t n = 1 << 20;
  float *buf = nullptr;
  if (hipMalloc(&buf, n * 4) != hipSuccess) return false;
  rabit::device::CheckHip(rabit::device::LaunchFill(buf, n, 6, 3.0, dev->stream()), "fill");
  Status s = dev->Allreduce(buf, buf, nullptr, n, 6, 2, 0, 1.0, nullptr);
  if (s == Status::kSuccess) s = dev->Finish(nullptr);
  std::vector<float> host(n);
  if (hipMemcpy(host.data(), buf, n * 4, hipMemcpyDeviceToHost) != hipSuccess) s = Status::kAborted;
  (void)hipFree(buf);
  bool ok = s == Status::kSuccess;
  for (size_t i = 0; i < n && ok; ++i) ok = host[i] == 3.0f;
  return ok;
}
}  // namespace

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);  // progress survives a kill by the test's time limit
  DevicePlane::ConfigureRcclEnv();  // as the engine does before starting threads
  DeviceConfig cfg;
  cfg.device = 0;
  cfg.comm_init_timeout_sec = 5;
  cfg.drain_timeout_sec = 10;
  DevicePlane dev(cfg, 0);
  hipStream_t st;
  rabit::device::CheckHip(hipStreamCreate(&st), "hipStreamCreate");
  dev.SetUserStream(st);

  // 1. rank 1 never joins: the deadline ends the init
  {
    printf("[1] init of a 2-rank communicator, rank 1 absent (deadline 5 s)...\n");
    const double t0 = Now();
    const Status s = dev.InitComm(DevicePlane::NewUniqueId(), 2, 0, nullptr);
    const double dt = Now() - t0;
    printf("[1] never-joining peer: status %s after %.2f s (deadline 5 s)\n",
           rabit::net::StatusName(s), dt);
    CHECK_TRUE(s == Status::kTimeout, "status %s", rabit::net::StatusName(s));
    CHECK_TRUE(dt >= 4.5 && dt < 30, "took %.2f s", dt);
    CHECK_TRUE(!dev.has_comm(), "communicator kept after the abort");
    CHECK_TRUE(WorldOneWorks(&dev), "world-1 communicator after the aborted init");
  }
  // 2. the failure probe reports a dead peer after 0.5 s: aborted long before the deadline
  {
    printf("[2] init of a 2-rank communicator, probe fires after 0.5 s...\n");
    const double t0 = Now();
    const Status s = dev.InitComm(DevicePlane::NewUniqueId(), 2, 0,
                                  [t0]() { return Now() - t0 > 0.5; });
    const double dt = Now() - t0;
    printf("[2] probe-detected failure: status %s after %.2f s\n", rabit::net::StatusName(s), dt);
    CHECK_TRUE(s == Status::kAborted, "status %s", rabit::net::StatusName(s));
    CHECK_TRUE(dt < 4.0, "took %.2f s", dt);
    CHECK_TRUE(!dev.has_comm(), "communicator kept after the abort");
    CHECK_TRUE(WorldOneWorks(&dev), "world-1 communicator after the probe abort");
  }
  // 3. an RCCL enqueue error is recoverable: kAborted, communicator dropped, next epoch works
  {
    DeviceConfig mc = cfg;
    mc.mock_rccl_error = 1;  // the first RCCL collective of this plane fails
    DevicePlane mdev(mc, 0);
    mdev.SetUserStream(st);
    const Status init = mdev.InitComm(DevicePlane::NewUniqueId(), 1, 0, nullptr);
    CHECK_TRUE(init == Status::kSuccess, "init %s", rabit::net::StatusName(init));
    mdev.BeginEpoch(1, 0);
    float *buf = nullptr;
    rabit::device::CheckHip(hipMalloc(&buf, 4096 * 4), "hipMalloc");
    const Status s = mdev.Allreduce(buf, buf, nullptr, 4096, 6, 2, 0, 1.0, nullptr);
    printf("[3] injected ncclRemoteError: status %s, communicator %s, aborts %llu\n",
           rabit::net::StatusName(s), mdev.has_comm() ? "kept" : "dropped",
           static_cast<unsigned long long>(mdev.rccl_aborts()));
    CHECK_TRUE(s == Status::kAborted, "status %s", rabit::net::StatusName(s));
    CHECK_TRUE(!mdev.has_comm() && mdev.rccl_aborts() == 1, "communicator not aborted");
    CHECK_TRUE(WorldOneWorks(&mdev), "next epoch after the injected error");
    (void)hipFree(buf);
  }
  // 4. abandoned bring-ups are bounded: cases 1 and 2 left two helpers blocked in RCCL's
  //    bootstrap; three more multi-rank bring-ups are refused at once instead of adding helpers
  {
    printf("[4] live abandoned helpers before: %d (cap %d)\n", DevicePlane::LiveAbandonedInits(),
           DevicePlane::kMaxAbandonedInits);
    CHECK_TRUE(DevicePlane::LiveAbandonedInits() == DevicePlane::kMaxAbandonedInits,
               "live %d", DevicePlane::LiveAbandonedInits());
    for (int i = 0; i < 3; ++i) {
      const double t0 = Now();
      const Status s = dev.InitComm(DevicePlane::NewUniqueId(), 2, 0, nullptr);
      const double dt = Now() - t0;
      printf("[4] bring-up %d: status %s after %.2f s, live abandoned %d\n", i,
             rabit::net::StatusName(s), dt, DevicePlane::LiveAbandonedInits());
      CHECK_TRUE(s == Status::kAborted && dt < 1.0, "status %s after %.2f s",
                 rabit::net::StatusName(s), dt);
      CHECK_TRUE(DevicePlane::LiveAbandonedInits() <= DevicePlane::kMaxAbandonedInits,
                 "live %d", DevicePlane::LiveAbandonedInits());
    }
    CHECK_TRUE(dev.init_refused() == 3, "refused %llu",
               static_cast<unsigned long long>(dev.init_refused()));
    CHECK_TRUE(WorldOneWorks(&dev), "world-1 communicator after the refused bring-ups");
  }
  printf("rccl_lifecycle_test: %s (%d failures); nonblocking settles %llu\n",
         g_fail ? "FAILED" : "OK", g_fail, static_cast<unsigned long long>(dev.rccl_settled()));
  fflush(stdout);
  return g_fail ? 1 : 0;
}
