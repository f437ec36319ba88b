// Flag semantics of the C++ drop-in (include/harp_amd/disort.hpp, DESIGN.md
// section 1): constructs harp_amd::Disort with each flag string given on the
// command line and prints "OK <flags>" or "REJECT <flags>: <message>".  Module
// construction runs only reset() (host code), so this runs without a GPU;
// tests/test_library.py::test_cpp_flag_semantics compares the verdicts with
// pyharp_amd.disort.check_flags.
#include <harp_amd/disort.hpp>

#include <cstdio>
#include <string>

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    harp_amd::DisortOptions op;
    op.header("flags").flags(argv[i]).nwave(1).ncol(1);
    op.ds().nlyr = 4;
    op.ds().nstr = 8;
    op.ds().nmom = 8;
    try {
      harp_amd::Disort disort(op);
      std::printf("OK %s\n", argv[i]);
    } catch (const c10::Error& e) {
      std::string msg = e.what_without_backtrace();
      std::printf("REJECT %s: %s\n", argv[i], msg.substr(0, msg.find('\n')).c_str());
    }
  }
  return 0;
}
