/*!
 * \file broadcast.cc
 * \brief Broadcast a string from node 0 (the reference's guide/broadcast.cc demo).
 */
#include <rabit/rabit.h>

#include <cstdio>
#include <string>

int main(int argc, char *argv[]) {
  rabit::Init(argc, argv);
  std::string s;
  if (rabit::GetRank() == 0) s = "hello world";
  printf("@node[%d] before-broadcast: s=\"%s\"\n", rabit::GetRank(), s.c_str());
  rabit::Broadcast(&s, 0);
  printf("@node[%d] after-broadcast: s=\"%s\"\n", rabit::GetRank(), s.c_str());
  rabit::Finalize();
  return 0;
}
