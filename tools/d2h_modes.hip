// Which D2H hipMemcpyAsync runs on a DMA engine and which as a blit kernel: run one mode per
// process under rocprofv3 --kernel-trace --memory-copy-trace.
//   plain   copy on a fresh non-blocking stream
//   xwait   the copy stream first waits on an event recorded on another stream (the checkpoint
//           mirror waits for its snapshot this way)
//   after   a kernel (memset) on the same stream right before the copy
//   lowprio xwait on a lowest-priority stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "plain";
  const size_t bytes = size_t(64) << 20;
  void *dev = nullptr, *host = nullptr;
  CK(hipMalloc(&dev, bytes));
  CK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
  hipStream_t main_s, side;
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  if (!std::strcmp(mode, "lowprio")) {
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, least));
  } else {
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  }
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int rep = 0; rep < 4; ++rep) {
    if (!std::strcmp(mode, "xwait") || !std::strcmp(mode, "lowprio")) {
      CK(hipMemsetAsync(dev, rep, bytes, main_s));
      CK(hipEventRecord(ev, main_s));
      CK(hipStreamWaitEvent(side, ev, 0));
    } else if (!std::strcmp(mode, "after")) {
      CK(hipMemsetAsync(dev, rep, bytes, side));
    }
    CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, side));
    CK(hipStreamSynchronize(side));
  }
  std::printf("{\"mode\":\"%s\",\"first_byte\":%d}\n", mode, static_cast<unsigned char *>(host)[0]);
  return 0;
}
