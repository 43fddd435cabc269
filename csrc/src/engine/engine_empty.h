/*!
 * \file engine_empty.h
 * \brief Single-process no-op engine (parity: reference `src/engine_empty.cc:17-141`).
 *        Collectives only run the lazy prepare function; rank 0, world size 1.
 */
#ifndef XRABIT_ENGINE_ENGINE_EMPTY_H_
#define XRABIT_ENGINE_ENGINE_EMPTY_H_

#include <string>

#include "rabit/internal/engine.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {

class EngineEmpty : public IEngine {
 public:
  bool Init(int, char **) { return true; }
  bool Shutdown() { return true; }
  void Allgather(void *, size_t, size_t, size_t, size_t, const char *, const int,
                 const char *) override {}
  void Allreduce(void *, size_t, size_t, ReduceFunction, PreprocFunction prepare_fun,
                 void *prepare_arg, const char *, const int, const char *) override {
    if (prepare_fun != nullptr) prepare_fun(prepare_arg);
  }
  void Broadcast(void *, size_t, int, const char *, const int, const char *) override {}
  void InitAfterException() override {}
  int LoadCheckPoint(Serializable *, Serializable *) override { return 0; }
  void CheckPoint(const Serializable *, const Serializable *) override { version_number_ += 1; }
  void LazyCheckPoint(const Serializable *) override { version_number_ += 1; }
  int VersionNumber() const override { return version_number_; }
  int GetRingPrevRank() const override { return 0; }
  int GetRank() const override { return 0; }
  int GetWorldSize() const override { return 1; }
  bool IsDistributed() const override { return false; }
  std::string GetHost() const override { return std::string(); }
  void TrackerPrint(const std::string &msg) override { utils::Printf("%s", msg.c_str()); }
  const char *EngineName() const override { return "empty"; }

 private:
  int version_number_{0};
};
}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ENGINE_EMPTY_H_
