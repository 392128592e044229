// Driver (ours) around the REFERENCE parallel_cpu_decomp.cpp, compiled from the
// reference's own source by oracle/Makefile.  The reference hard-codes one OpenMP
// thread (`int thread_count = 1;`, parallel_cpu_decomp.cpp:24, applied at :634); this
// driver sets it from argv[1] and runs the reference's own main() unchanged.
//   decomp_driver <threads>       (reads data.bin in the working directory)
#define main reference_decomp_main
#include "parallel_cpu_decomp.cpp"
#undef main

#include <cstdlib>

int main(int argc, char** argv) {
  if (argc > 1 && std::atoi(argv[1]) > 0) thread_count = std::atoi(argv[1]);
  return reference_decomp_main(argc, argv);
}
