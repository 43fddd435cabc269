/*!
 * \file lazy_allreduce.cc
 * \brief Lazy preparation (the reference's guide/lazy_allreduce.cc demo): the prepare
 *        lambda fills the buffer right before the reduction and is skipped when the result
 *        is recovered from peers after a failure (try it with the mock engine).
 */
#include <rabit/rabit.h>

#include <cstdio>

int main(int argc, char *argv[]) {
  const int n = 3;
  int a[n] = {0, 0, 0};
  rabit::Init(argc, argv);
  const int rank = rabit::GetRank();
  auto prepare = [&]() {
    printf("@node[%d] run prepare function\n", rank);
    for (int i = 0; i < n; ++i) a[i] = rank + i;
  };
  printf("@node[%d] before-allreduce: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Allreduce<rabit::op::Max>(&a[0], n, prepare);
  printf("@node[%d] after-allreduce-max: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Allreduce<rabit::op::Sum>(&a[0], n);
  printf("@node[%d] after-allreduce-sum: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Finalize();
  return 0;
}
