// Range-split feasibility model (round 4): decode a 4 MiB generator block as R
// independent output ranges and count the matches whose bytes depend on an
// earlier range (taint spreads through the sources of later matches).
// g++ -O2 -Iinclude -o /tmp/taint tools/taint_sim.cpp bo-lz4-ada_amd/csrc/lz4gen.cpp
// /tmp/taint <kind 0 dense|1 mixed> <R ranges> <log2 granule>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string.h>
extern "C" int64_t lz4ada_gen_block(int kind, uint64_t seed, uint8_t* raw, int64_t raw_len, uint8_t* comp, int64_t comp_cap);
struct S { int64_t ipos, lit, L, off, ml, dst; };
int main(int argc, char** argv) {
  int kind = atoi(argv[1]); int R = atoi(argv[2]); int G = atoi(argv[3]);
  int64_t n = 4 << 20; std::vector<uint8_t> raw(n), comp(n * 2);
  double tot_tb = 0, tot_tm = 0, tot_seq = 0, tot_gb=0, tot_gm=0, tot_depth=0; int nb = 8;
  for (int b = 0; b < nb; ++b) {
    int64_t cl = lz4ada_gen_block(kind, 1000 + b, raw.data(), n, comp.data(), comp.size());
    std::vector<S> seqs; int64_t p = 0, o = 0;
    while (p < cl) { S s; s.ipos = p; int tk = comp[p++]; int64_t L = tk >> 4; if (L == 15) { int e; do { e = comp[p++]; L += e; } while (e == 255); }
      s.lit = p; s.L = L; p += L; s.dst = o; o += L; if (p >= cl) { s.off = 0; s.ml = 0; seqs.push_back(s); break; }
      s.off = comp[p] | (comp[p+1] << 8); p += 2; int64_t M = tk & 15; if (M == 15) { int e; do { e = comp[p++]; M += e; } while (e == 255); }
      s.ml = M + 4; s.dst = o; o += s.ml; seqs.push_back(s); }
    // ranges by compressed position
    std::vector<uint8_t> taint(o, 0), gt((o >> 4) + 2, 0);  // exact, granule
    std::vector<int> depth(o, 0);
    for (int r = 1; r < R; ++r) {
      int64_t cut = cl * r / R; cut &= ~int64_t(16383);
      // find first seq with ipos >= cut
      size_t i = 0; while (i < seqs.size() && seqs[i].ipos < cut) ++i;
      int64_t ostart = seqs[i].dst - seqs[i].L; // literal start
      int64_t oend = o; if (r + 1 < R) { int64_t c2 = (cl * (r+1) / R) & ~int64_t(16383); size_t j = i; while (j < seqs.size() && seqs[j].ipos < c2) ++j; oend = seqs[j].dst - seqs[j].L; }
      int64_t tb = 0, tm = 0, gb = 0, gm = 0, md = 0;
      for (size_t j = i; j < seqs.size(); ++j) { const S& s = seqs[j]; if (s.dst >= oend) break; if (!s.ml) continue;
        int64_t src = s.dst - s.off; bool t = false, tg = false; int d = 0;
        for (int64_t k = 0; k < s.ml; ++k) { int64_t q = src + (k % s.off); if (q < ostart) { t = true; d = d > 1 ? d : 1; } else if (taint[q]) { t = true; d = d > depth[q]+1 ? d : depth[q]+1; } }
        int64_t qe = src + (s.off < s.ml ? s.off : s.ml);
        for (int64_t q = (src >> G) ; q <= ((qe - 1) >> G); ++q) { if ((q << G) < ostart || gt[q]) tg = true; }
        if (t) { tm++; tb += s.ml; for (int64_t k = 0; k < s.ml; ++k) { taint[s.dst + k] = 1; depth[s.dst+k] = d; } if (d > md) md = d; }
        if (tg) { gm++; gb += s.ml; for (int64_t q = s.dst >> G; q <= ((s.dst + s.ml - 1) >> G); ++q) gt[q] = 1; }
      }
      tot_tb += tb; tot_tm += tm; tot_gb += gb; tot_gm += gm; tot_depth += md;
    }
    tot_seq += seqs.size();
  }
  printf("kind %d R %d G %d: seqs/block %.0f  exact tainted matches/block %.0f bytes %.0f | granule matches %.0f bytes %.0f | max depth avg %.1f\n", kind, R, 1<<G, tot_seq/nb, tot_tm/nb, tot_tb/nb, tot_gm/nb, tot_gb/nb, tot_depth/nb);
}
