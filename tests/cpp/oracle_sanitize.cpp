// Drives the CPU oracle (oracle/oracle.cpp, linked in directly) under AddressSanitizer +
// UndefinedBehaviorSanitizer: all 8 reference scenes, all 3 variants, the
// pixel-list render in both accumulation orders, ray queries, the sampler and the mesh BVH
// builder.  Writes every result to argv[1] as raw floats so tests/test_oracle_sanitize.py can
// check them against the normal (unsanitized) oracle build bit for bit.
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
void* orc_scene_build(int scene_id, float light_intensity);
void orc_scene_free(void* h);
int orc_scene_n_prims(void* h);
int orc_scene_depth(void* h);
int orc_scene_export(void* h, float* prims, float* nodes, int* leaves);
void orc_camera(int W, int H, float* invPV, float* invV);
int orc_render(const float* prims, int n_prims, const float* nodes, const int* leaves, int depth,
               const float* invPV, const float* invV, int W, int H, int first_pass, int n_passes, float date,
               int bounces, float ior, int variant, int row_step, int row_offset, int n_threads, float* accum,
               unsigned long long* events, unsigned* trav_px, const void* meshes);
int orc_render_pixels(const float* prims, int n_prims, const float* nodes, const int* leaves, int depth,
                      const float* invPV, const float* invV, int W, int H, const int* xy, int n_px, int first_pass,
                      int n_passes, float date, int bounces, float ior, int variant, int per_pass, int n_threads,
                      float* acc);
int orc_trace(const float* prims, int n_prims, const float* nodes, const int* leaves, int depth,
              const float* origins, const float* dirs, int n, int any_hit, int prim, int* out_i, float* out_f,
              const void* meshes);
void orc_sample_hemisphere(const float* normal3, const float* fseed3, float roughness, int nb_used, int n,
                           float* out);
int orc_mesh_bvh(const float* verts, const int* tris, int n_tris, float* nodes_out, int* leaves_out);
}

static std::vector<float> out;
static void emit(const float* p, size_t n) { out.insert(out.end(), p, p + n); }

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int W = 16, H = 12;
  float ipv[16], iv[16];
  orc_camera(W, H, ipv, iv);
  for (int s = 1; s <= 8; ++s) {
    void* sc = orc_scene_build(s, 1.2f);
    if (!sc) return 3;
    const int n = orc_scene_n_prims(sc), d = orc_scene_depth(sc);
    std::vector<float> prims((size_t)n * 64), nodes((size_t)((2 << d) - 1) * 6);
    std::vector<int> leaves((size_t)1 << d);
    orc_scene_export(sc, prims.data(), nodes.data(), leaves.data());
    const int B = s == 1 ? 3 : (s == 8 ? 12 : 8);
    for (int variant = 0; variant < 3; ++variant) {
      if (variant > 0 && s != 6) continue;
      std::vector<float> acc((size_t)W * H * 3, 0.0f);
      unsigned long long ev[11] = {0};
      if (orc_render(prims.data(), n, nodes.data(), leaves.data(), d, ipv, iv, W, H, 1, 2, 0.0f, B,
                     s == 6 ? 1.5f : 1.0f, variant, 1, 0, 2, acc.data(), ev, nullptr, nullptr) != 0)
        return 4;
      emit(acc.data(), acc.size());
    }
    const int xy[6] = {0, 0, 7, 5, 15, 11};
    for (int per_pass = 0; per_pass < 2; ++per_pass) {
      float px[9] = {0};
      if (orc_render_pixels(prims.data(), n, nodes.data(), leaves.data(), d, ipv, iv, W, H, xy, 3, 5, 40, 0.0f, B,
                            1.0f, 0, per_pass, 2, px) != 0)
        return 5;
      emit(px, 9);
    }
    const float O[6] = {0.0f, -347.0f, 61.0f, 10.0f, 20.0f, 30.0f};
    const float D[6] = {0.0f, 0.98f, -0.17f, 0.3f, -0.5f, -0.8f};
    for (int any = 0; any < 2; ++any) {
      int oi[6];
      float of[42];
      if (orc_trace(prims.data(), n, nodes.data(), leaves.data(), d, O, D, 2, any, -1, oi, of, nullptr) != 0) return 6;
      emit(of, 42);
    }
    orc_scene_free(sc);
  }
  const float nrm[3] = {0.2f, 0.3f, 0.9f}, seed[3] = {0.25f, 3.5f, 0.75f};
  float pts[3 * 64];
  orc_sample_hemisphere(nrm, seed, 0.7f, 3, 64, pts);
  emit(pts, 3 * 64);
  // a small mesh: a 4x4 grid of quads (32 triangles)
  std::vector<float> verts;
  std::vector<int> tris;
  for (int j = 0; j < 5; ++j)
    for (int i = 0; i < 5; ++i) { verts.push_back((float)i); verts.push_back((float)j); verts.push_back(0.1f * (float)(i * j)); }
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 4; ++i) {
      const int a = j * 5 + i;
      tris.insert(tris.end(), {a, a + 1, a + 5, a + 1, a + 6, a + 5});
    }
  std::vector<float> mnodes(63 * 6);
  std::vector<int> mleaves(32);
  const int md = orc_mesh_bvh(verts.data(), tris.data(), 32, mnodes.data(), mleaves.data());
  if (md != 5) return 7;
  emit(mnodes.data(), mnodes.size());
  FILE* f = std::fopen(argv[1], "wb");
  if (!f) return 8;
  std::fwrite(out.data(), sizeof(float), out.size(), f);
  std::fclose(f);
  std::printf("oracle sanitize run: %zu floats\n", out.size());
  return 0;
}
