// chol_plan_check.hip — host-only check of the split Cholesky's task table
// (chol_split_plan, bundleadjustment_amd/csrc/ba_chol_split.hip): replays the
// launches of every block step and asserts that each tile (I, J) receives
// every panel p < J exactly once, in order and in time (before panel J /
// diagonal block J is formed), only once the panel exists, and that no two
// tasks of one launch touch one tile.  Prints the per-step work of one order.
//   hipcc --offload-arch=gfx950 -O1 -std=c++17 -I bundleadjustment_amd/csrc \
//         tools/chol_plan_check.hip -o /tmp/chol_plan_check && /tmp/chol_plan_check [T] [rank] [budget]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "ba_chol_split.hip"

using namespace bahip;

static int check(int T, int TR, int rank, double budget, bool show) {
  CholSplitPlan P;
  chol_split_plan(T, TR, rank, budget, P);
  std::vector<std::vector<int>> a(TR, std::vector<int>(T, 0));   // panels applied, in order
  int bad = 0;
  auto fail = [&](const char* what, int k, int I, int J, int x) {
    if (bad++ < 10) printf("T=%d TR=%d rank %d step %d: tile (%d,%d) %s (%d)\n", T, TR, rank, k, I, J, what, x);
  };
  for (int k = 0; k + 1 < T; ++k) {
    for (int I = k + 1; I < TR; ++I)
      if (a[I][k] != k) fail("panel formed before all updates", k, I, k, a[I][k]);
    if (a[k + 1][k + 1] != k) fail("critical: diagonal not at panel k", k, k + 1, k + 1, a[k + 1][k + 1]);
    std::vector<std::vector<int>> touch(TR, std::vector<int>(T, 0));
    touch[k + 1][k + 1] = 1;
    a[k + 1][k + 1] = k + 1;
    long work = 0;
    for (int t = P.off[k]; t < P.off[k + 1]; ++t) {
      const int4 q = P.tasks[t];
      const int I = q.x & 0xfffff, J = q.y;
      if (I < J || I >= TR || J >= T || J < 1) { fail("outside the trapezoid", k, I, J, 0); continue; }
      if (touch[I][J]++) fail("two tasks in one launch", k, I, J, 0);
      if (q.z != a[I][J]) fail("range does not continue the applied prefix", k, I, J, q.z);
      if ((q.w <= q.z && !(q.x >> 20)) || q.w > k + 1) fail("panel range empty or not formed yet", k, I, J, q.w);
      if (q.w > (I == J ? J - 1 : J)) fail("range beyond the tile's panels", k, I, J, q.w);
      if (((q.x >> 20) & 1) != (J == k + 1 && I > J)) fail("column-task mark", k, I, J, q.x >> 20);
      a[I][J] = q.w;
      work += q.w - q.z;
    }
    if (show)
      printf("step %3d: %5d tasks, %6ld panel-tile updates\n", k, P.off[k + 1] - P.off[k], work);
  }
  for (int J = 1; J < T; ++J)
    for (int I = J; I < TR; ++I)
      if (a[I][J] != J) fail("end: not every panel applied", T, I, J, a[I][J]);
  return bad;
}

// the flow form's one list: replay it in order with the chain workgroup
// advancing whenever its inputs are complete (step k: tiles (k+1, k) and
// (k+1, k+1) at panel k), and check that every task's inputs are complete
// when it comes (tile prefix, panels, V) — a task that needs a V the chain
// cannot produce from the tasks before it could hold the last free slot
static int check_flow(int T, int TR, int rank) {
  CholSplitPlan P;
  chol_split_plan(T, TR, rank, 1.0, P);
  std::vector<int4> flow;
  chol_flow_tasks(P.tasks, P.off, flow);
  std::vector<std::vector<int>> a(TR, std::vector<int>(T, 0));
  std::vector<std::vector<char>> pan(TR, std::vector<char>(T, 0));
  std::vector<char> V(T, 0);
  for (int I = 1; I < TR; ++I) pan[I][0] = 1;   // panel 0: before the launch
  V[0] = 1;
  int chain = 0;                                // next step of the chain workgroup
  auto advance = [&]() {
    while (chain + 1 < T && a[chain + 1][chain] == chain && a[chain + 1][chain + 1] == chain) {
      a[chain + 1][chain + 1] = chain + 1;      // (the chain applies panel k to the diagonal itself)
      V[chain + 1] = 1;
      ++chain;
    }
  };
  int bad = 0;
  auto fail = [&](const char* what, int i, int x, int y) {
    if (bad++ < 10) printf("flow T=%d TR=%d rank %d: entry %d (%d,%d): %s\n", T, TR, rank, i, x, y, what);
  };
  if (flow.size() != P.tasks.size()) fail("layout", 0, 0, 0);
  advance();
  for (int i = 0; i < (int)flow.size(); ++i) {
    const int4 q = flow[i];
    const int I = q.x & 0xfffff, J = q.y;
    if (a[I][J] != q.z) fail("tile prefix", i, I, J);
    for (int p = q.z; p < q.w; ++p)
      if (!pan[I][p] || !pan[J][p]) fail("panel not formed", i, I, J);
    a[I][J] = q.w;
    if ((q.x >> 20) & 1) {
      advance();
      if (!V[J]) fail("V not reachable by the chain", i, I, J);
      if (a[I][J] != J) fail("column task: tile incomplete", i, I, J);
      pan[I][J] = 1;
    }
    advance();
  }
  if (chain != T - 1) fail("chain did not finish", 0, chain, T);
  return bad;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "quick") {   // (tests/test_chol_plan.py: T <= 40)
    int bad = 0, cases = 0;
    for (int rank : {1, 4})
      for (int T = 2; T <= 40; ++T)
        for (int TR = T; TR <= T + 1; ++TR, ++cases) bad += check(T, TR, rank, 1.0, false) + check_flow(T, TR, rank);
    printf("%d cases, %d violations\n", cases, bad);
    return bad ? 1 : 0;
  }
  if (argc > 1) {
    const int T = atoi(argv[1]);
    return check(T, T, argc > 2 ? atoi(argv[2]) : 4, argc > 3 ? atof(argv[3]) : 1.0, true) ? 1 : 0;
  }
  int bad = 0, cases = 0;
  for (int rank = 1; rank <= 8; rank *= 2)
    for (double budget : {0.5, 1.0, 1.5})
      for (int T = 2; T <= 100; ++T)
        for (int TR = T; TR <= T + 1; ++TR, ++cases) bad += check(T, TR, rank, budget, false);
  for (int T = 2; T <= 100; ++T)
    for (int TR = T; TR <= T + 1; ++TR, ++cases) bad += check_flow(T, TR, 4);
  printf("%d cases, %d violations\n", cases, bad);
  return bad ? 1 : 0;
}
