// ba_options.cpp — ba_default_options (include/ba_hip.h): the options of
// BAOptimizer::configureSolver (ba_project/src/ba/Optimizer.cpp:80-90) plus
// the Ceres defaults it leaves in place.  Plain host C++: compiled into
// libba_hip.so and, for the ASan/UBSan build of the shim (tests/cpp
// `make sanitize`), into the oracle-backed driver.
#include "ba_hip.h"

extern "C" void ba_default_options(ba_options* o) {
  if (!o) return;
  o->max_num_iterations = 50;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->linear_solver = BA_DENSE_SCHUR;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->preconditioner_type = BA_JACOBI;
  o->max_linear_solver_iterations = 500;
  o->min_linear_solver_iterations = 0;
  o->precision = BA_FP64;
  o->eta = 1e-1;
}
