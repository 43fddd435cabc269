/*!
 * \file broadcast.cc
 * \brief Broadcast (semantics of the reference's guide/broadcast.cc): rank 0 owns a string and a
 *        small parameter vector; after rabit::Broadcast every rank holds both.  Strings and
 *        std::vector are sized on the root and resized on the receivers by the API.
 */
#include <rabit/rabit.h>

#include <cstdio>
#include <string>
#include <vector>

int main(int argc, char *argv[]) {
  rabit::Init(argc, argv);
  const int me = rabit::GetRank();
  const bool root = me == 0;
  std::string greeting = root ? "hello world" : "";
  std::vector<float> params;
  if (root) params = {0.5f, 1.5f, 2.5f};
  std::printf("@node[%d] before-broadcast: s=\"%s\" (%zu params)\n", me, greeting.c_str(),
              params.size());
  rabit::Broadcast(&greeting, 0);
  rabit::Broadcast(&params, 0);
  std::printf("@node[%d] after-broadcast: s=\"%s\" (%zu params, sum %.1f)\n", me,
              greeting.c_str(), params.size(),
              params.empty() ? 0.0 : params[0] + params[1] + params[2]);
  rabit::Finalize();
  return 0;
}
