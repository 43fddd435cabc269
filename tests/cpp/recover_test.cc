/*!
 * \file recover_test.cc
 * \brief Multi-process recovery scenarios, run under rabit_amd.launcher with mock kill points.
 *
 * Covers the intent of the reference's test/model_recover.cc, local_recover.cc and
 * lazy_recover.cc in one program:
 *   mode=global  CheckPoint(global) ; Max (lazy prepare), Broadcast from several roots, Sum,
 *                Allgather, all verified against closed forms
 *   mode=local   CheckPoint(global, local): the local model is replicated on the ring
 *   mode=lazy    LazyCheckPoint(global)
 * With rabit_bootstrap_cache=1 a bootstrap Allreduce<Max> runs before LoadCheckPoint.
 * Usage: recover_test <ndata> mode=<global|local|lazy> [niter=3] [rabit params...]
 */
#include <rabit/c_api.h>
#include <rabit/rabit.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
struct VecModel : public rabit::Serializable {
  std::vector<float> v;
  void Load(rabit::Stream *fi) override { rabit::utils::Check(fi->Read(&v), "load model"); }
  void Save(rabit::Stream *fo) const override { fo->Write(v); }
};

// contribution of rank r to element i at iteration it (integers: exact in fp32)
inline float Contrib(size_t i, int r, int modulus, float base) {
  return static_cast<float>((i * static_cast<size_t>(r + 1)) % static_cast<size_t>(modulus)) +
         base;
}

std::string Arg(int argc, char **argv, const char *key, const char *dflt) {
  const size_t k = strlen(key);
  for (int i = 1; i < argc; ++i) {
    if (strncmp(argv[i], key, k) == 0 && argv[i][k] == '=') return argv[i] + k + 1;
  }
  return dflt;
}
}  // namespace

int main(int argc, char *argv[]) {
  if (argc < 2) {
    printf("Usage: recover_test <ndata> mode=<global|local|lazy> [niter=N] [params]\n");
    return 0;
  }
  const size_t n = static_cast<size_t>(atol(argv[1]));
  const std::string mode = Arg(argc, argv, "mode", "global");
  const int niter = atoi(Arg(argc, argv, "niter", "3").c_str());
  rabit::Init(argc, argv);
  const int rank = rabit::GetRank();
  const int world = rabit::GetWorldSize();

  // collective issued before LoadCheckPoint: only replayable with rabit_bootstrap_cache=1
  if (Arg(argc, argv, "rabit_bootstrap_cache", "0") != "0") {
    int top = rank;
    rabit::Allreduce<rabit::op::Max>(&top, 1);
    rabit::utils::Check(top == world - 1, "[%d] bootstrap max rank %d != %d", rank, top,
                        world - 1);
  }

  VecModel global, local;
  const bool use_local = mode == "local";
  int start = use_local ? rabit::LoadCheckPoint(&global, &local) : rabit::LoadCheckPoint(&global);
  if (start == 0) {
    global.v.assign(n, 1.0f);
    if (use_local) local.v.assign(n, 1.0f + rank);
  }
  printf("[%d] start at version %d (engine %s)\n", rank, start,
         rabit::engine::GetEngine()->EngineName());
  fflush(stdout);

  for (int it = start; it < niter; ++it) {
    // base value of rank r for element i: local mode keeps local = global + rank
    auto base = [&](size_t i, int r) { return global.v[i] + (use_local ? r : 0); };
    // ---- Max with a lazy prepare function (skipped when the result is replayed)
    {
      const int z = 111 + it;
      std::vector<float> buf(n);
      rabit::Allreduce<rabit::op::Max>(buf.data(), n, [&]() {
        for (size_t i = 0; i < n; ++i) {
          buf[i] = Contrib(i, rank, z, use_local ? local.v[i] : global.v[i]);
        }
      });
      for (size_t i = 0; i < n; ++i) {
        float expect = Contrib(i, 0, z, base(i, 0));
        for (int r = 1; r < world; ++r) expect = std::max(expect, Contrib(i, r, z, base(i, r)));
        rabit::utils::Check(buf[i] == expect, "[%d] Max mismatch at %zu: %f vs %f", rank, i,
                            buf[i], expect);
      }
    }
    // ---- Broadcast a string from several roots
    {
      const int stride = std::max(world / 3, 1);
      for (int root = 0; root < world; root += stride) {
        std::string expect(n, '\0');
        for (size_t i = 0; i < n; ++i) expect[i] = static_cast<char>((i + root) % 126 + 1);
        std::string got;
        if (rank == root) got = expect;
        rabit::Broadcast(&got, root);
        rabit::utils::Check(got == expect, "[%d] Broadcast from %d mismatch", rank, root);
      }
    }
    // ---- Sum; the result becomes the next global model
    std::vector<float> sum(n);
    {
      const int z = 131 + it;
      for (size_t i = 0; i < n; ++i) {
        sum[i] = Contrib(i, rank, z, use_local ? local.v[i] : global.v[i]);
      }
      rabit::Allreduce<rabit::op::Sum>(sum.data(), n);
      for (size_t i = 0; i < n; ++i) {
        float expect = 0;
        for (int r = 0; r < world; ++r) expect += Contrib(i, r, z, base(i, r));
        rabit::utils::Check(std::fabs(sum[i] - expect) < 1e-5f, "[%d] Sum mismatch at %zu",
                            rank, i);
      }
    }
    // ---- Allgather of per-rank slices
    if (mode == "global") {
      const int z = 151 + it;
      std::vector<float> all(n * world);
      for (size_t i = 0; i < n; ++i) all[rank * n + i] = Contrib(i, rank, z, global.v[i]);
      rabit::Allgather(all.data(), all.size(), rank * n, n, n);  // begin, size, prev size
      for (int r = 0; r < world; ++r) {
        for (size_t i = 0; i < n; ++i) {
          rabit::utils::Check(all[r * n + i] == Contrib(i, r, z, global.v[i]),
                              "[%d] Allgather mismatch slice %d", rank, r);
        }
      }
    }
    for (size_t i = 0; i < n; ++i) global.v[i] = std::fmod(sum[i], 1000.0f);
    if (use_local) {
      for (size_t i = 0; i < n; ++i) local.v[i] = global.v[i] + rank;
      rabit::CheckPoint(&global, &local);
    } else if (mode == "lazy") {
      rabit::LazyCheckPoint(&global);
    } else {
      rabit::CheckPoint(&global);
    }
    printf("[%d] iteration %d done (version %d)\n", rank, it, rabit::VersionNumber());
    fflush(stdout);
  }
  // transports used (extension of the C API): {"n_shm_ops":...} etc.
  const std::string stats = RabitGetStats();
  const size_t at = stats.find("\"n_shm_ops\":");
  const long shm_ops = at == std::string::npos ? -1 : atol(stats.c_str() + at + 12);
  rabit::Finalize();
  printf("[%d] PASSED shm_ops=%ld\n", rank, shm_ops);
  return 0;
}
