// chol_plan_check.hip — host-only check of the grouped split Cholesky's task
// schedule (chol_upd_plan, bundleadjustment_amd/csrc/ba_chol_split.hip):
// replays the launches of every block step and asserts that each tile (I, J)
// receives every panel p < J exactly once, in time (before panel J / diagonal
// block J is formed), and that no two tasks of one launch touch one tile.
//   hipcc --offload-arch=gfx950 -O1 -std=c++17 -I bundleadjustment_amd/csrc \
//         tools/chol_plan_check.hip -o /tmp/chol_plan_check && /tmp/chol_plan_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "ba_chol_split.hip"

using namespace bahip;

static int check(int T, int TR) {
  // got[I][J] = bitmask of panels applied (T <= 128: two words)
  std::vector<std::vector<std::vector<char>>> got(TR, std::vector<std::vector<char>>(T, std::vector<char>(T, 0)));
  int bad = 0;
  auto need_all = [&](int I, int J, int upto, int k, const char* what) {
    for (int p = 0; p < upto; ++p)
      if (got[I][J][p] != 1) {
        if (bad++ < 10) printf("T=%d TR=%d step %d: tile (%d,%d) has panel %d x%d at %s\n", T, TR, k, I, J, p, got[I][J][p], what);
      }
  };
  for (int k = 0; k + 1 < T; ++k) {
    // panel k: A_{I,k}, I > k, must hold panels < k
    for (int I = k + 1; I < TR; ++I) need_all(I, k, k, k, "panel");
    const CholUpd u = chol_upd_plan(k, T, TR);
    std::vector<std::vector<int>> touch(TR, std::vector<int>(T, 0));
    // critical: diagonal k + 1 takes panel k, must hold panels < k
    need_all(k + 1, k + 1, k, k, "critical");
    touch[k + 1][k + 1]++;
    got[k + 1][k + 1][k]++;
    for (int s = 0; s < u.nseg; ++s) {
      const CholUpdSeg& g = u.seg[s];
      int cnt = 0;
      for (int J = g.ja; J < g.jb; ++J) {
        const int c = upd_col_tiles(g, J, TR);
        for (int b = 0; b < c; ++b, ++cnt) {
          const int I = g.diag ? J : J + (J == g.xd ? 1 : 0) + b;
          if (I >= TR || I < J) { if (bad++ < 10) printf("bad tile (%d,%d)\n", I, J); continue; }
          touch[I][J]++;
          for (int p = g.pa; p < g.pb; ++p) got[I][J][p]++;
        }
      }
      if (cnt != g.cnt) { if (bad++ < 10) printf("T=%d step %d seg %d count %d vs %d\n", T, k, s, cnt, g.cnt); }
    }
    for (int I = 0; I < TR; ++I)
      for (int J = 0; J < T; ++J)
        if (touch[I][J] > 1 && bad++ < 10) printf("T=%d step %d: tile (%d,%d) written by %d tasks\n", T, k, I, J, touch[I][J]);
  }
  // at the end every tile (I, J), J < T, holds every panel p < J exactly once
  for (int J = 0; J < T; ++J)
    for (int I = J; I < TR; ++I) need_all(I, J, J, T, "end");
  return bad;
}

int main() {
  int bad = 0, cases = 0;
  for (int T = 2; T <= 100; ++T)
    for (int TR = T; TR <= T + 1; ++TR, ++cases) bad += check(T, TR);
  printf("%d cases, %d violations\n", cases, bad);
  return bad ? 1 : 0;
}
