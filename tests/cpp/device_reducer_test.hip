/*!
 * \file device_reducer_test.hip
 * \brief rabit::DeviceReducer on HBM and host buffers: an (argmax value, index) struct reducer
 *        and a 24-byte moment accumulator, checked against closed forms.
 *        usage: device_reducer_test [n] [rabit params...]
 */
#include <hip/hip_runtime.h>
#include <rabit/device_reducer.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

struct ArgMax {
  float v;
  int idx;
};
struct ArgMaxOp {
  __host__ __device__ void operator()(ArgMax &dst, const ArgMax &src) const {
    if (src.v > dst.v || (src.v == dst.v && src.idx < dst.idx)) dst = src;
  }
};
struct Moments {  // 24 bytes: not a power of two
  double sum, sumsq;
  long long cnt;
};
struct MomentsOp {
  __host__ __device__ void operator()(Moments &dst, const Moments &src) const {
    dst.sum += src.sum;
    dst.sumsq += src.sumsq;
    dst.cnt += src.cnt;
  }
};

#define CHECK_HIP(x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                          \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

static float Val(size_t i, int r) { return static_cast<float>((i * 7 + r * 13) % 101); }

int main(int argc, char *argv[]) {
  size_t n = 100003;
  if (argc > 1 && atol(argv[1]) > 0) n = static_cast<size_t>(atol(argv[1]));
  rabit::Init(argc, argv);
  const int rank = rabit::GetRank(), world = rabit::GetWorldSize();
  const int dev = rabit::GetDevice();
  if (dev < 0) {
    fprintf(stderr, "no device plane\n");
    return 3;
  }
  CHECK_HIP(hipSetDevice(dev));
  std::vector<ArgMax> h(n);
  std::vector<Moments> m(n);
  for (size_t i = 0; i < n; ++i) {
    h[i] = ArgMax{Val(i, rank), static_cast<int>(i % 100000) * world + rank};
    m[i] = Moments{static_cast<double>(rank + i % 3), static_cast<double>((rank + 1) * (rank + 1)),
                   1};
  }
  ArgMax *dh = nullptr;
  Moments *dm = nullptr;
  CHECK_HIP(hipMalloc(&dh, n * sizeof(ArgMax)));
  CHECK_HIP(hipMalloc(&dm, n * sizeof(Moments)));
  CHECK_HIP(hipMemcpy(dh, h.data(), n * sizeof(ArgMax), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(dm, m.data(), n * sizeof(Moments), hipMemcpyHostToDevice));
  rabit::DeviceReducer<ArgMax, ArgMaxOp> argmax;
  rabit::DeviceReducer<Moments, MomentsOp> moments;
  int prepared = 0;
  argmax.Allreduce(dh, n, [&]() { ++prepared; });
  moments.Allreduce(dm, n);
  argmax.Allreduce(h.data(), n);  // host buffer: host form of the same functor
  std::vector<ArgMax> gd(n);
  std::vector<Moments> gm(n);
  CHECK_HIP(hipMemcpy(gd.data(), dh, n * sizeof(ArgMax), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(gm.data(), dm, n * sizeof(Moments), hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) {
    ArgMax want{-1.0f, 0};
    for (int r = 0; r < world; ++r) {
      ArgMax c{Val(i, r), static_cast<int>(i % 100000) * world + r};
      ArgMaxOp()(want, c);
    }
    double s = 0, q = 0;
    for (int r = 0; r < world; ++r) {
      s += r + i % 3;
      q += (r + 1) * (r + 1);
    }
    if (gd[i].v != want.v || gd[i].idx != want.idx) ++bad;
    if (h[i].v != want.v || h[i].idx != want.idx) ++bad;
    if (gm[i].sum != s || gm[i].sumsq != q || gm[i].cnt != world) ++bad;
  }
  CHECK_HIP(hipFree(dh));
  CHECK_HIP(hipFree(dm));
  rabit::Finalize();
  // the lazy prepare runs exactly once, or not at all on a restarted worker whose first
  // collective was recovered from the survivors
  const char *att = getenv("DMLC_NUM_ATTEMPT");
  const bool restarted = att != nullptr && atoi(att) > 0;
  if (bad != 0 || prepared > 1 || (prepared == 0 && !restarted)) {
    fprintf(stderr, "[%d] DEVREDUCER FAILED: %zu mismatches, prepare ran %d times\n", rank, bad,
            prepared);
    return 1;
  }
  printf("[%d] DEVREDUCER OK (n=%zu, world=%d)\n", rank, n, world);
  return 0;
}
