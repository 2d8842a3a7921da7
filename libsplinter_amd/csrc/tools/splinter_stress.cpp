// MRSW stress bench: 1 writer + (threads-1) readers on a hot key set
// (reference /root/reference/splinter_stress.c; defaults :274-294).
#include "stress_common.hpp"

int main(int argc, char** argv) {
  stress::Config c;
#ifdef SPLINTER_PERSISTENT
  c.slots = 25000; c.max_value = 2048; c.threads = 16; c.duration_ms = 30000; c.keys = 10000;
#endif
  for (int i = 1; i < argc; ++i)
    if (!stress::parse_common(c, argc, argv, i)) { stress::usage(argv[0]); return 2; }
  c.lanes = false;
  const bool mrsw = c.writers == 1;
  return stress::run(c, mrsw ? "MRSW" : "MRMW-SHARED", mrsw ? "readers + 1 writer" : "readers + shared-key writers");
}
