// Driver (ours) around the REFERENCE parallel_cpu_prescan.cpp, compiled from the
// reference's own source by oracle/Makefile.  The reference hard-codes its OpenMP
// thread count (`int thread_count = 16;`, parallel_cpu_prescan.cpp:25, applied at
// :593); this driver sets it from argv[1] (e.g. nproc) and then runs the reference's
// own main() unchanged (same input file, same timing and verification lines).
//   prescan_driver <threads>      (reads data100_100.bin in the working directory)
#define main reference_prescan_main
#include "parallel_cpu_prescan.cpp"
#undef main

#include <cstdlib>

int main(int argc, char** argv) {
  if (argc > 1 && std::atoi(argv[1]) > 0) thread_count = std::atoi(argv[1]);
  return reference_prescan_main(argc, argv);
}
