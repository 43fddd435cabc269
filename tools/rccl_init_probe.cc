// Step-by-step probe of a non-blocking RCCL communicator init that can never complete (rank 1
// of 2 never joins): which call blocks, and does ncclCommAbort return?  Diagnostic only.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int blocking = argc > 1 ? atoi(argv[1]) : 0;
  const double t0 = Now();
  hipSetDevice(0);
  ncclUniqueId id;
  printf("%.3f getUniqueId...\n", Now() - t0);
  ncclResult_t r = ncclGetUniqueId(&id);
  printf("%.3f getUniqueId -> %d\n", Now() - t0, r);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = blocking;
  ncclComm_t comm = nullptr;
  printf("%.3f initRankConfig(nranks=2, rank=0, blocking=%d)...\n", Now() - t0, blocking);
  r = ncclCommInitRankConfig(&comm, 2, id, 0, &cfg);
  printf("%.3f initRankConfig -> %d comm=%p\n", Now() - t0, r, (void *)comm);
  for (int i = 0; i < 30; ++i) {
    ncclResult_t st = ncclSuccess;
    printf("%.3f getAsyncError...\n", Now() - t0);
    ncclResult_t q = ncclCommGetAsyncError(comm, &st);
    printf("%.3f getAsyncError -> %d state %d\n", Now() - t0, q, st);
    if (st != ncclInProgress) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
  }
  printf("%.3f abort...\n", Now() - t0);
  r = ncclCommAbort(comm);
  printf("%.3f abort -> %d\n", Now() - t0, r);
  return 0;
}
