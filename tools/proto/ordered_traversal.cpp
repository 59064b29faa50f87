// Prototype / analysis (never part of the product): does a front-to-back BVH traversal
// (nearer child popped first, cull at push AND at pop time) return the same closest-hit
// record as the reference's DFS (right child first, cull at push only,
// raytracer_func.frag:734-769), and how many node visits does it save?
//
// Built against the oracle itself (#include of oracle.cpp): every traversal of an oracle
// render is replayed with the ordered walk through oracle's analysis hook and the two hit
// records (prim, shape, face, dist, pl, pg) are compared bit for bit.
//
//   g++ -O2 -std=c++17 -ffp-contract=off -mfma -pthread -o /tmp/ordered tools/proto/ordered_traversal.cpp
//   /tmp/ordered SCENE W H PASSES BOUNCES
#include "../../oracle/oracle.cpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>

namespace orc {

static std::atomic<unsigned long long> g_trav{0}, g_mismatch{0}, g_nodes_ref{0}, g_nodes_ord{0};
static std::atomic<unsigned long long> g_leaves_ord{0}, g_popcull{0};

// intersect_bv with the cull distance returned instead of compared (same arithmetic)
static bool box_entry(const Ctx& c, int i, V3 O, V3 D, float* dist) {
  const float* nd = c.sc.nodes + (size_t)i * 6;
  V3 bmin = v3(nd[0], nd[1], nd[2]), bmax = v3(nd[3], nd[4], nd[5]);
  V3 center = v3((bmin.x + bmax.x) / 2.0f, (bmin.y + bmax.y) / 2.0f, (bmin.z + bmax.z) / 2.0f);
  V3 width = v3(0.5f * (bmax.x - bmin.x), 0.5f * (bmax.y - bmin.y), 0.5f * (bmax.z - bmin.z));
  V3 iw = v3(1.0f / width.x, 1.0f / width.y, 1.0f / width.z);
  V3 Oi = (O - center) * iw;
  V3 Di = D * iw;
  if (fabsf(Oi.x) < 1.0f && fabsf(Oi.y) < 1.0f && fabsf(Oi.z) < 1.0f) { *dist = 0.0f; return true; }
  float al = FLT_MAXV;
  float rD[3] = {(1.0f / D.x) * width.x, (1.0f / D.y) * width.y, (1.0f / D.z) * width.z};
  float oi[3] = {Oi.x, Oi.y, Oi.z}, di[3] = {Di.x, Di.y, Di.z};
  for (int f = 0; f < 6; ++f) {
    int c0 = f / 2;
    if (fabsf(di[c0]) > EPSILON) {
      int c1 = (c0 + 1) % 3, c2 = (c0 + 2) % 3;
      float cd = -1.0f + 2.0f * (float)(f % 2);
      float a = (cd - oi[c0]) * rD[c0];
      if ((a > EPSILON) && (fabsf(oi[c1] + a * di[c1]) <= 1.0f) && (fabsf(oi[c2] + a * di[c2]) <= 1.0f))
        if (a < al) al = a;
    }
  }
  if (al < FLT_MAXV) {
    V3 Pg = (al * Di + Oi) * width + center;
    *dist = distance3(O, Pg);
    return true;
  }
  return false;
}

static void ordered_walk(Ctx& c, V3 O, V3 D, unsigned long long* nodes, unsigned long long* leaves,
                         unsigned long long* popcull) {
  int st[64];
  float sd[64];
  int head = 1;
  st[0] = 0; sd[0] = 0.0f;
  reset_inter(c);
  const int leaf0 = (1 << c.sc.depth) - 1;
  while (head > 0) {
    head--;
    const int i = st[head];
    if (sd[head] > c.ci.dist) { ++*popcull; continue; }
    if (i >= leaf0) {
      ++*leaves;
      const int p = c.sc.leaves[i - leaf0];
      if (p >= 0) intersect_prim(c, p, O, D);
    } else {
      ++*nodes;
      const int j = 2 * i + 1;
      float dl = 0.0f, dr = 0.0f;
      const bool hl = box_entry(c, j, O, D, &dl) && dl <= c.ci.dist;
      const bool hr = box_entry(c, j + 1, O, D, &dr) && dr <= c.ci.dist;
      if (hl && hr) {
        if (dr <= dl) { st[head] = j; sd[head++] = dl; st[head] = j + 1; sd[head++] = dr; }
        else { st[head] = j + 1; sd[head++] = dr; st[head] = j; sd[head++] = dl; }
      } else if (hl) { st[head] = j; sd[head++] = dl; }
      else if (hr) { st[head] = j + 1; sd[head++] = dr; }
    }
  }
}

static thread_local unsigned long long tl_nodes_ref_prev = 0;

static void hook(const Ctx& c, V3 O, V3 D) {
  Ctx o = c;
  unsigned long long n = 0, l = 0, pc = 0;
  ordered_walk(o, O, D, &n, &l, &pc);
  g_trav++;
  g_nodes_ord += n;
  g_leaves_ord += l;
  g_popcull += pc;
  g_nodes_ref += c.ev[EV_NODE] - tl_nodes_ref_prev;
  tl_nodes_ref_prev = c.ev[EV_NODE];
  const Hit& a = c.ci;
  const Hit& b = o.ci;
  const bool same = a.shape == b.shape && a.index == b.index && a.dir == b.dir &&
                    (a.shape < 0 || (fbits(a.dist) == fbits(b.dist) && fbits(a.pl.x) == fbits(b.pl.x) &&
                                     fbits(a.pl.y) == fbits(b.pl.y) && fbits(a.pl.z) == fbits(b.pl.z) &&
                                     fbits(a.pg.x) == fbits(b.pg.x) && fbits(a.pg.y) == fbits(b.pg.y) &&
                                     fbits(a.pg.z) == fbits(b.pg.z)));
  if (!same) {
    if (g_mismatch++ < 5)
      fprintf(stderr, "mismatch: ref (shape %d prim %d dist %.9g) ordered (shape %d prim %d dist %.9g)\n", a.shape,
              a.index, a.dist, b.shape, b.index, b.dist);
  }
}

}  // namespace orc

int main(int argc, char** argv) {
  const int sid = argc > 1 ? atoi(argv[1]) : 8;
  const int W = argc > 2 ? atoi(argv[2]) : 192, H = argc > 3 ? atoi(argv[3]) : 108;
  const int S = argc > 4 ? atoi(argv[4]) : 8, B = argc > 5 ? atoi(argv[5]) : 8;
  void* h = orc_scene_build(sid, 1.2f);
  const int n = orc_scene_n_prims(h), d = orc_scene_depth(h);
  std::vector<float> prims((size_t)n * 64), nodes((size_t)((2 << d) - 1) * 6);
  std::vector<int> leaves((size_t)1 << d);
  orc_scene_export(h, prims.data(), nodes.data(), leaves.data());
  float ipv[16], iv[16];
  orc_camera(W, H, ipv, iv);
  std::vector<float> acc((size_t)W * H * 3, 0.0f);
  unsigned long long ev[16] = {0};
  orc::g_trav_hook = orc::hook;
  orc_render(prims.data(), n, nodes.data(), leaves.data(), d, ipv, iv, W, H, 1, S, 0.0f, B, 1.0f, 0, 1, 0, 8,
             acc.data(), ev, nullptr, nullptr);
  const double t = (double)orc::g_trav.load();
  printf("{\"scene\": %d, \"W\": %d, \"H\": %d, \"spp\": %d, \"B\": %d, \"traversals\": %.0f, \"mismatches\": %llu, "
         "\"node_visits_ref\": %.3f, \"node_visits_ordered\": %.3f, \"leaf_visits_ordered\": %.3f, "
         "\"pop_culls\": %.3f}\n",
         sid, W, H, S, B, t, orc::g_mismatch.load(), orc::g_nodes_ref.load() / t, orc::g_nodes_ord.load() / t,
         orc::g_leaves_ord.load() / t, orc::g_popcull.load() / t);
  orc_scene_free(h);
  return 0;
}
