/*!
 * \file basic.cc
 * \brief What Allreduce does (the reference's guide/basic.cc demo): each node holds
 *        a[i] = rank + i; Max then Sum across nodes.
 */
#include <rabit/rabit.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char *argv[]) {
  const int n = argc > 1 ? atoi(argv[1]) : 3;
  std::vector<int> a(n);
  rabit::Init(argc, argv);
  const int rank = rabit::GetRank();
  for (int i = 0; i < n; ++i) a[i] = rank + i;
  printf("@node[%d] before-allreduce: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Allreduce<rabit::op::Max>(a.data(), n);
  printf("@node[%d] after-allreduce-max: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Allreduce<rabit::op::Sum>(a.data(), n);
  printf("@node[%d] after-allreduce-sum: a={%d, %d, %d}\n", rank, a[0], a[1], a[2]);
  rabit::Finalize();
  return 0;
}
