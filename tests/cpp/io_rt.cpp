// io_rt.cpp — round trip through the C++ problem I/O header
// (bundleadjustment_amd/host/ba_io.hpp): BAS load -> save, BAL text -> BAS.
// Built plain by tests/test_io.py and with ASan + UBSan by `make sanitize`.
#include <cstdio>

#include "ba_io.hpp"

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s in.bas out.bas in_bal.txt out_bal.bas\n", argv[0]);
    return 2;
  }
  try {
    ba_amd::ProblemData p = ba_amd::load_problem(argv[1]);
    ba_amd::save_problem(argv[2], p);
    ba_amd::ProblemData b = ba_amd::read_bal(argv[3], 2.0, false);
    ba_amd::save_problem(argv[4], b);
    ba_problem v = p.view();
    std::printf("%d %d %d\n", v.n_cams, v.n_pts, v.n_obs);
  } catch (const std::exception& e) {
    std::printf("error: %s\n", e.what());
    return 1;
  }
  return 0;
}
