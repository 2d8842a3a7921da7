// MRMW "chi sao" bench: W writers on disjoint key lanes + readers over the
// whole key space (reference /root/reference/splinter_chi_sao.c, lanes :400-418,
// MAX_WRITERS 32 :29).
#include "stress_common.hpp"

int main(int argc, char** argv) {
  stress::Config c;
  c.writers = 4;
  for (int i = 1; i < argc; ++i)
    if (!stress::parse_common(c, argc, argv, i)) { stress::usage(argv[0]); return 2; }
  if (c.writers > 32) c.writers = 32;
  c.lanes = true;
  return stress::run(c, "MRMW", "readers + disjoint-lane writers");
}
