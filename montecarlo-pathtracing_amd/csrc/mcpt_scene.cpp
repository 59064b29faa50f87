// mcpt_scene.cpp — host-side scene producer of the hot path (C++, no GL, no Eigen).
//
// Restates the reference's host pipeline that feeds the sampling loop:
//   * Transfo::translate/scale/rotateX/Y/Z in degrees   easycppogl/gl_eigen.cpp:29-105
//   * Material / PrimData (256 B = 16 RGBA32F texels)    bvh_gpu/scene.h:30-73
//   * ScenePrimitives::add_* with areas, prim_bb         scene.h:128-172, scene.cpp:18-53
//   * sortEmissiveFirst (non-stable partition)           scene.cpp:70-88
//   * BVH_KDtree median splits (std::nth_element, x→y→z) bvh.cpp:5-93
//   * BVH_GPU_Scene::finalize → flat buffers             gpu_bvh_scene.cpp:121-187
//   * the 8 scene builders                               MontecarloGPU/montecarlo.cpp:629-795
//   * the canonical camera                               easycppogl/camera.cpp:53-95
// Float products follow Eigen's lazy coefficient product without FMA (SSE4 build of the
// reference, CMakeLists.txt -msse4): res(i,j) = ((a_i0 b_0j + a_i1 b_1j) + a_i2 b_2j) + a_i3 b_3j.
// Compiled with -ffp-contract=off.  The 4x4 inverse is evaluated in double and rounded
// (Eigen's SSE float inverse is not reproducible without Eigen).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/mcpt.h"

// mcpt_capi.hip: an error return without a detail (drops the thread's unread detail)
int mcpt_err_bare(int status);

namespace mcpt {
namespace host {

struct Mat4 {
  float m[16];   // column-major
  float& operator()(int r, int c) { return m[c * 4 + r]; }
  float operator()(int r, int c) const { return m[c * 4 + r]; }
  static Mat4 identity() {
    Mat4 a;
    std::memset(a.m, 0, sizeof(a.m));
    a(0, 0) = a(1, 1) = a(2, 2) = a(3, 3) = 1.0f;
    return a;
  }
  Mat4 operator*(const Mat4& b) const {
    Mat4 r;
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 4; ++i) {
        float acc = (*this)(i, 0) * b(0, j);
        for (int k = 1; k < 4; ++k) acc = acc + (*this)(i, k) * b(k, j);
        r(i, j) = acc;
      }
    return r;
  }
  void apply(const float in[4], float out[4]) const {
    for (int i = 0; i < 4; ++i) {
      float acc = (*this)(i, 0) * in[0];
      for (int k = 1; k < 4; ++k) acc = acc + (*this)(i, k) * in[k];
      out[i] = acc;
    }
  }
  Mat4 inverse() const;
};

Mat4 Mat4::inverse() const {
  // adjugate / determinant in double, cofactors in the classic expanded form
  const float* a = m;
  auto A = [&](int i) { return (double)a[i]; };
  double c[16];
  c[0] = A(5) * A(10) * A(15) - A(5) * A(11) * A(14) - A(9) * A(6) * A(15) + A(9) * A(7) * A(14) + A(13) * A(6) * A(11) - A(13) * A(7) * A(10);
  c[4] = -A(4) * A(10) * A(15) + A(4) * A(11) * A(14) + A(8) * A(6) * A(15) - A(8) * A(7) * A(14) - A(12) * A(6) * A(11) + A(12) * A(7) * A(10);
  c[8] = A(4) * A(9) * A(15) - A(4) * A(11) * A(13) - A(8) * A(5) * A(15) + A(8) * A(7) * A(13) + A(12) * A(5) * A(11) - A(12) * A(7) * A(9);
  c[12] = -A(4) * A(9) * A(14) + A(4) * A(10) * A(13) + A(8) * A(5) * A(14) - A(8) * A(6) * A(13) - A(12) * A(5) * A(10) + A(12) * A(6) * A(9);
  c[1] = -A(1) * A(10) * A(15) + A(1) * A(11) * A(14) + A(9) * A(2) * A(15) - A(9) * A(3) * A(14) - A(13) * A(2) * A(11) + A(13) * A(3) * A(10);
  c[5] = A(0) * A(10) * A(15) - A(0) * A(11) * A(14) - A(8) * A(2) * A(15) + A(8) * A(3) * A(14) + A(12) * A(2) * A(11) - A(12) * A(3) * A(10);
  c[9] = -A(0) * A(9) * A(15) + A(0) * A(11) * A(13) + A(8) * A(1) * A(15) - A(8) * A(3) * A(13) - A(12) * A(1) * A(11) + A(12) * A(3) * A(9);
  c[13] = A(0) * A(9) * A(14) - A(0) * A(10) * A(13) - A(8) * A(1) * A(14) + A(8) * A(2) * A(13) + A(12) * A(1) * A(10) - A(12) * A(2) * A(9);
  c[2] = A(1) * A(6) * A(15) - A(1) * A(7) * A(14) - A(5) * A(2) * A(15) + A(5) * A(3) * A(14) + A(13) * A(2) * A(7) - A(13) * A(3) * A(6);
  c[6] = -A(0) * A(6) * A(15) + A(0) * A(7) * A(14) + A(4) * A(2) * A(15) - A(4) * A(3) * A(14) - A(12) * A(2) * A(7) + A(12) * A(3) * A(6);
  c[10] = A(0) * A(5) * A(15) - A(0) * A(7) * A(13) - A(4) * A(1) * A(15) + A(4) * A(3) * A(13) + A(12) * A(1) * A(7) - A(12) * A(3) * A(5);
  c[14] = -A(0) * A(5) * A(14) + A(0) * A(6) * A(13) + A(4) * A(1) * A(14) - A(4) * A(2) * A(13) - A(12) * A(1) * A(6) + A(12) * A(2) * A(5);
  c[3] = -A(1) * A(6) * A(11) + A(1) * A(7) * A(10) + A(5) * A(2) * A(11) - A(5) * A(3) * A(10) - A(9) * A(2) * A(7) + A(9) * A(3) * A(6);
  c[7] = A(0) * A(6) * A(11) - A(0) * A(7) * A(10) - A(4) * A(2) * A(11) + A(4) * A(3) * A(10) + A(8) * A(2) * A(7) - A(8) * A(3) * A(6);
  c[11] = -A(0) * A(5) * A(11) + A(0) * A(7) * A(9) + A(4) * A(1) * A(11) - A(4) * A(3) * A(9) - A(8) * A(1) * A(7) + A(8) * A(3) * A(5);
  c[15] = A(0) * A(5) * A(10) - A(0) * A(6) * A(9) - A(4) * A(1) * A(10) + A(4) * A(2) * A(9) + A(8) * A(1) * A(6) - A(8) * A(2) * A(5);
  double det = A(0) * c[0] + A(1) * c[4] + A(2) * c[8] + A(3) * c[12];
  Mat4 r;
  for (int i = 0; i < 16; ++i) r.m[i] = (float)(c[i] / det);
  return r;
}

namespace xf {   // easycppogl/gl_eigen.cpp:29-105
Mat4 T(float x, float y, float z) { Mat4 a = Mat4::identity(); a(0, 3) = x; a(1, 3) = y; a(2, 3) = z; return a; }
Mat4 S(float x, float y, float z) { Mat4 a = Mat4::identity(); a(0, 0) = x; a(1, 1) = y; a(2, 2) = z; return a; }
Mat4 S(float s) { return S(s, s, s); }
static inline float deg2rad(float a) { return (float)(M_PI / 180) * a; }
Mat4 Rx(float deg) { float t = deg2rad(deg), s = std::sin(t), c = std::cos(t); Mat4 a = Mat4::identity(); a(1, 1) = c; a(2, 1) = s; a(1, 2) = -s; a(2, 2) = c; return a; }
Mat4 Ry(float deg) { float t = deg2rad(deg), s = std::sin(t), c = std::cos(t); Mat4 a = Mat4::identity(); a(0, 0) = c; a(2, 0) = -s; a(0, 2) = s; a(2, 2) = c; return a; }
Mat4 Rz(float deg) { float t = deg2rad(deg), s = std::sin(t), c = std::cos(t); Mat4 a = Mat4::identity(); a(0, 0) = c; a(1, 0) = s; a(0, 1) = -s; a(1, 1) = c; return a; }
}  // namespace xf

struct Material {
  float rgba[4];
  float shininess, roughness, emissivity;
};

enum PrimCode { kMesh = 0, kSphere = 1, kCube = 2, kCylinder = 3, kCone = 4, kQuad = 5 };

struct Vec3 { float x, y, z; };
static Vec3 sub(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static Vec3 cross(Vec3 a, Vec3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static float sqnorm(Vec3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static float norm(Vec3 a) { return std::sqrt(sqnorm(a)); }
static Vec3 apply_pt(const Mat4& t, float x, float y, float z) {
  float in[4] = {x, y, z, 1.0f}, o[4];
  t.apply(in, o);
  return {o[0], o[1], o[2]};
}

static void kd_build(const std::vector<Vec3>& centre, const std::vector<float>& box, int& depth,
                     std::vector<float>& nodes, std::vector<int>& leaves);

// PrimData record (scene.h:64-73) + the BVH built over the records
class PrimScene {
 public:
  std::vector<float> records;   // 64 floats per primitive
  std::vector<float> nodes;     // (2^(d+1)-1) × 6
  std::vector<int> leaves;      // 2^d
  int depth = 0, nb_emissive = 0;
  bool finalized = false;

  int count() const { return (int)(records.size() / 64); }
  float* rec(int i) { return records.data() + (size_t)i * 64; }
  const float* rec(int i) const { return records.data() + (size_t)i * 64; }

  void clear() {
    records.clear(); nodes.clear(); leaves.clear(); meshes.clear();
    depth = 0; nb_emissive = 0; finalized = false;
  }

  int push(int code, const Mat4& trf, const Material& mat, float area) {   // scene.cpp:44-53
    Mat4 inv = trf.inverse();
    size_t base = records.size();
    records.resize(base + 64, 0.0f);
    float* r = records.data() + base;
    std::memcpy(r, trf.m, 64);
    std::memcpy(r + 16, inv.m, 64);
    std::memcpy(r + 32, trf.m, 64);
    r[48] = (float)code;
    std::memcpy(r + 52, mat.rgba, 16);
    r[56] = mat.shininess; r[57] = mat.roughness; r[58] = mat.emissivity; r[59] = area;
    finalized = false;
    return count() - 1;
  }
  void box_edges(const Mat4& t, Vec3& U, Vec3& V, Vec3& W) const {
    Vec3 o = apply_pt(t, -1, -1, -1);
    U = sub(apply_pt(t, 1, -1, -1), o);
    V = sub(apply_pt(t, -1, 1, -1), o);
    W = sub(apply_pt(t, -1, -1, 1), o);
  }
  int sphere(const Mat4& t, const Material& m) {
    float r = norm(Vec3{t(0, 0), t(1, 0), t(2, 0)});
    return push(kSphere, t, m, (float)(2.0 * M_PI) * r * r);
  }
  int cube(const Mat4& t, const Material& m) {
    Vec3 U, V, W; box_edges(t, U, V, W);
    return push(kCube, t, m, 2.0f * ((norm(cross(U, V)) + norm(cross(U, W))) + norm(cross(W, V))));
  }
  int cylinder(const Mat4& t, const Material& m) {
    Vec3 U, V, W; box_edges(t, U, V, W);
    return push(kCylinder, t, m, (((sqnorm(U) + sqnorm(V)) / 4.0f) * std::sqrt(2.0f)) * (float)M_PI * norm(W));
  }
  int cone(const Mat4& t, const Material& m) { return push(kCone, t, m, 0.0f); }
  int quad(const Mat4& t, const Material& m) {
    Vec3 o = apply_pt(t, -1, -1, 0);
    Vec3 U = sub(apply_pt(t, 1, -1, 0), o), V = sub(apply_pt(t, -1, 1, 0), o);
    return push(kQuad, t, m, norm(cross(U, V)));
  }

  // ScenePrimitives::prim_bb: AABB of the transformed ±1.005 cube (quads: z = ±0.001)
  Vec3 prim_box(int p, float* bb) const {
    const float* r = rec(p);
    Mat4 t; std::memcpy(t.m, r, 64);
    float lo[3] = {3.40282347e38f, 3.40282347e38f, 3.40282347e38f};
    float hi[3] = {-3.40282347e38f, -3.40282347e38f, -3.40282347e38f};
    for (uint32_t corner = 0; corner < 8; ++corner) {
      float c[4] = {(float)(corner & 1) * 2.01f - 1.005f, (float)(corner >> 1 & 1) * 2.01f - 1.005f,
                    (float)(corner >> 2 & 1) * 2.01f - 1.005f, 1.0f};
      if (r[48] == 5.0f) c[2] /= std::fabs(c[2]) * 1000.0f;
      float w[4];
      t.apply(c, w);
      for (int k = 0; k < 3; ++k) {
        if (w[k] < lo[k]) lo[k] = w[k];
        if (w[k] > hi[k]) hi[k] = w[k];
      }
    }
    for (int k = 0; k < 3; ++k) { bb[k] = lo[k]; bb[3 + k] = hi[k]; }
    return Vec3{(lo[0] + hi[0]) / 2.0f, (lo[1] + hi[1]) / 2.0f, (lo[2] + hi[2]) / 2.0f};
  }

  int emissive_first() {   // scene.cpp:70-88 — swap-based, non-stable (order matters for the BVH)
    int n = count(), head = 0;
    while (head < n && rec(head)[58] > 0.0f) ++head;
    std::vector<float> tmp(64);
    for (int i = head; i < n; ++i) {
      if (rec(i)[58] > 0.0f) {
        std::memcpy(tmp.data(), rec(head), 256);
        std::memcpy(rec(head), rec(i), 256);
        std::memcpy(rec(i), tmp.data(), 256);
        ++head;
      }
    }
    return head;
  }

  int finalize() {   // BVH_GPU_Scene::finalize + BVH_KDtree::init/compute
    int n = count();
    if (n <= 0) return mcpt_err_bare(MCPT_ERR_BAD_SCENE);
    nb_emissive = emissive_first();
    std::vector<Vec3> centre(n);
    std::vector<float> box((size_t)n * 6);
    for (int i = 0; i < n; ++i) centre[i] = prim_box(i, &box[(size_t)i * 6]);
    kd_build(centre, box, depth, nodes, leaves);
    finalized = true;
    return MCPT_OK;
  }

  // ---- triangle meshes (BVH_GPU_Scene::add_mesh / place_mesh, gpu_bvh_scene.cpp:51-74,
  //      gpu_bvh_scene.h:89-92; ScenePrimitives::add_mesh scene.cpp:56-67)
  struct Mesh {
    std::vector<float> verts, normals;   // 3 per vertex
    std::vector<uint32_t> tris;          // 3 per triangle, mesh-local vertex indices
    float bbmin[3], bbmax[3];            // Mesh::BB()
    int depth = 0;
    std::vector<float> nodes;            // (2^(d+1)-1) × 6, mesh-local space
    std::vector<int> leaves;             // 2^d mesh-local triangle ids or -1
  };
  std::vector<Mesh> meshes;

  // SceneMesh::prim_bb (scene.cpp:106-122): triangle AABB grown by 0.001, its centre
  static Vec3 tri_box(const Mesh& m, int t, float* bb) {
    const float* P[3];
    for (int k = 0; k < 3; ++k) P[k] = &m.verts[(size_t)m.tris[(size_t)t * 3 + k] * 3];
    for (int i = 0; i < 3; ++i) {
      bb[i] = std::min({P[0][i], P[1][i], P[2][i]}) - 0.001f;
      bb[3 + i] = std::max({P[0][i], P[1][i], P[2][i]}) + 0.001f;
    }
    return Vec3{(bb[0] + bb[3]) / 2.0f, (bb[1] + bb[4]) / 2.0f, (bb[2] + bb[5]) / 2.0f};
  }

  int add_mesh(const float* v, const float* nrm, int nv, const uint32_t* t, int nt, const float* bb6) {
    if (!v || !nrm || !t || nv <= 0 || nt <= 0) return -1;
    for (int i = 0; i < nt * 3; ++i)
      if (t[i] >= (uint32_t)nv) return -1;
    Mesh m;
    m.verts.assign(v, v + (size_t)nv * 3);
    m.normals.assign(nrm, nrm + (size_t)nv * 3);
    m.tris.assign(t, t + (size_t)nt * 3);
    if (bb6) {
      for (int k = 0; k < 3; ++k) { m.bbmin[k] = bb6[k]; m.bbmax[k] = bb6[3 + k]; }
    } else {   // BoundingBox::add_point over the vertices (easycppogl/mesh.h:38-76)
      for (int k = 0; k < 3; ++k) { m.bbmin[k] = v[k]; m.bbmax[k] = v[k]; }
      for (int i = 1; i < nv; ++i)
        for (int k = 0; k < 3; ++k) {
          m.bbmin[k] = std::min(m.bbmin[k], v[(size_t)i * 3 + k]);
          m.bbmax[k] = std::max(m.bbmax[k], v[(size_t)i * 3 + k]);
        }
    }
    std::vector<Vec3> centre(nt);
    std::vector<float> box((size_t)nt * 6);
    for (int i = 0; i < nt; ++i) centre[i] = tri_box(m, i, &box[(size_t)i * 6]);
    kd_build(centre, box, m.depth, m.nodes, m.leaves);   // BVH_GPU_Scene::add_bvh → compute
    meshes.push_back(std::move(m));
    finalized = false;
    return (int)meshes.size() - 1;
  }

  // ScenePrimitives::add_mesh: transfo = trf · BB.matrix(), inverse = trf^-1, mesh transfo = trf,
  // type (0, mesh line) — the mesh id here; area 0
  int place_mesh(int mesh, const Mat4& trf, const Material& mat) {
    if (mesh < 0 || mesh >= (int)meshes.size()) return -1;
    const Mesh& m = meshes[mesh];
    const float c[3] = {(m.bbmin[0] + m.bbmax[0]) / 2.0f, (m.bbmin[1] + m.bbmax[1]) / 2.0f,
                        (m.bbmin[2] + m.bbmax[2]) / 2.0f};
    const float sc[3] = {(m.bbmax[0] - m.bbmin[0]) / 2.0f, (m.bbmax[1] - m.bbmin[1]) / 2.0f,
                         (m.bbmax[2] - m.bbmin[2]) / 2.0f};
    const Mat4 trBB = trf * (xf::T(c[0], c[1], c[2]) * xf::S(sc[0], sc[1], sc[2]));   // BoundingBox::matrix()
    int i = push(kMesh, trBB, mat, 0.0f);
    float* r = rec(i);
    const Mat4 inv = trf.inverse();
    std::memcpy(r + 16, inv.m, 64);
    std::memcpy(r + 32, trf.m, 64);
    r[49] = (float)mesh;
    return i;
  }
};

// BVH_KDtree::compute (bvh.cpp:34-93) over precomputed boxes / centres: ceil(log2 n) levels,
// depth-1 rounds of std::nth_element median splits on x → y → z, leaf pairs from the right
// (a lone item: left leaf + -1, its box twice), internal boxes merged bottom-up.
static void kd_build(const std::vector<Vec3>& centre, const std::vector<float>& box, int& depth,
                     std::vector<float>& nodes, std::vector<int>& leaves) {
  const int n = (int)centre.size();
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  depth = (int)std::ceil(std::log2((float)n));
  std::vector<int> bounds{0, n}, next;
  int axis = 0;
  for (int round = 1; round < depth; ++round) {
    next.assign(1, bounds[0]);
    for (size_t s = 1; s < bounds.size(); ++s) {
      int64_t lo = bounds[s - 1], hi = bounds[s], mid = (lo + hi) / 2;
      auto key = [&](int id) { return axis == 0 ? centre[id].x : (axis == 1 ? centre[id].y : centre[id].z); };
      std::nth_element(order.begin() + lo, order.begin() + mid, order.begin() + hi,
                       [&](int a, int b) { return key(a) < key(b); });
      next.push_back((int)mid);
      next.push_back((int)hi);
    }
    bounds.swap(next);
    axis = (axis + 1) % 3;
  }
  const int n_leaf = 1 << depth, n_node = 2 * n_leaf - 1;
  leaves.assign(n_leaf, -1);
  nodes.assign((size_t)n_node * 6, 0.0f);
  auto put = [&](int node, int item) { std::memcpy(&nodes[(size_t)node * 6], &box[(size_t)item * 6], 24); };
  if (n == 1) {
    put(0, 0);   // depth 0: the root is the only leaf and keeps id -1 (bvh.cpp writes ind[-1])
    return;
  }
  int node = n_node - 1, leaf = n_leaf - 1;
  for (int s = (int)bounds.size() - 1; s > 0; --s, node -= 2, leaf -= 2) {
    int first = bounds[s - 1];
    if (bounds[s] - first == 1) {
      int id = order[first];
      leaves[leaf] = -1; leaves[leaf - 1] = id;
      put(node, id); put(node - 1, id);
    } else {
      leaves[leaf] = order[first + 1]; put(node, order[first + 1]);
      leaves[leaf - 1] = order[first]; put(node - 1, order[first]);
    }
  }
  for (int k = n_node - 1; k >= 2; k -= 2) {   // merge (scene.cpp:91-100)
    float* parent = &nodes[(size_t)((k - 2) / 2) * 6];
    const float* c1 = &nodes[(size_t)k * 6];
    const float* c2 = &nodes[(size_t)(k - 1) * 6];
    for (int q = 0; q < 3; ++q) {
      parent[q] = std::min(c1[q], c2[q]);
      parent[3 + q] = std::max(c1[3 + q], c2[3 + q]);
    }
  }
}

// ------------------------------------------------------------------------------------
// the reference scenes (montecarlo.cpp:629-795); colours montecarlo.cpp:33-44
// ------------------------------------------------------------------------------------
namespace palette {
const float red[4] = {0.9f, 0, 0, 1}, green[4] = {0, 0.9f, 0, 1}, blue[4] = {0, 0, 0.9f, 1};
const float yellow[4] = {0.9f, 0.9f, 0, 1}, cyan[4] = {0, 0.9f, 0.9f, 1}, magenta[4] = {0.9f, 0, 0.9f, 1};
const float white[4] = {0.9f, 0.9f, 0.9f, 1}, black[4] = {0, 0, 0, 1};
}  // namespace palette

static Material mat(const float c[4], float shin = 0.0f, float rough = 0.0f, float emis = 0.0f, float opacity = -1.0f) {
  Material m;
  std::memcpy(m.rgba, c, 16);
  if (opacity >= 0.0f) m.rgba[3] = opacity;
  m.shininess = shin; m.roughness = rough; m.emissivity = emis;
  return m;
}
static Material rgba_mat(float r, float g, float b, float a, float shin, float rough) {
  float c[4] = {r, g, b, a};
  return mat(c, shin, rough);
}

using namespace xf;

// Menger sponge (montecarlo.cpp:143-179): 20 sub-cubes per level
static void sponge(PrimScene& sc, const Mat4& m, int d, float sc_factor, const Material& mt) {
  const float x = 2.0f / 3.0f, y = sc_factor / 3.0f;
  static const signed char kOffsets[20][3] = {
      {1, 1, 0}, {-1, 1, 0}, {-1, -1, 0}, {1, -1, 0}, {1, 0, 1}, {-1, 0, 1}, {-1, 0, -1},
      {1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, -1, -1}, {0, 1, -1}, {1, 1, 1}, {-1, 1, 1},
      {-1, -1, 1}, {1, -1, 1}, {1, 1, -1}, {-1, 1, -1}, {-1, -1, -1}, {1, -1, -1}};
  auto coord = [&](signed char k) { return k == 0 ? 0.0f : (k > 0 ? x : -x); };
  for (const auto& o : kOffsets) {
    Mat4 child = m * (T(coord(o[0]), coord(o[1]), coord(o[2])) * S(y));
    if (d > 0) sponge(sc, child, d - 1, sc_factor, mt);
    else sc.cube(child, mt);
  }
}

// floor, optional ceiling and back wall shared by the boxes of scenes 1, 2, 4
static void box_shell(PrimScene& sc, bool with_top) {
  using namespace palette;
  sc.quad(T(0, 0, -100) * S(100, 100, 1), mat(white));
  if (with_top) sc.quad(T(0, 0, 100) * Rx(180) * S(100, 100, 1), mat(white));
  sc.quad(T(0, 100, 0) * Rx(90) * S(100, 100, 1), mat(cyan));
}

static int build_reference(PrimScene& sc, int id, float li) {
  using namespace palette;
  sc.clear();
  switch (id) {
    case 1:   // scene_box_diffuse (key Q)
      box_shell(sc, true);
      sc.quad(T(0, -100, 0) * Rx(-90) * S(100, 100, 1), mat(yellow));
      sc.quad(T(-100, 0, 0) * Ry(90) * S(100, 100, 1), mat(red));
      sc.quad(T(100, 0, 0) * Ry(-90) * S(100, 100, 1), mat(green));
      sc.cube(T(70, 20, -40) * Rz(20) * S(20, 20, 60), mat(white));
      sc.cube(T(-70, 40, -40) * Rz(-20) * S(20, 20, 60), mat(white));
      sc.quad(T(0, 0, 99) * Rx(180) * S(40, 40, 1), mat(white, 0, 0, 10 * li));
      break;
    case 2:   // scene_box_balls (key W)
    case 4: { // scene_box_no_top (key R)
      const bool balls = (id == 2);
      box_shell(sc, balls);
      sc.quad(T(0, 99, 0) * Rx(90) * S(40, 60, 1), mat(white, 1, 1));
      sc.quad(T(0, -100, 0) * Rx(-90) * S(100, 100, 1), mat(white));
      sc.quad(T(-100, 0, 0) * Ry(90) * S(100, 100, 1), mat(white));
      sc.quad(T(100, 0, 0) * Ry(-90) * S(100, 100, 1), mat(white));
      sc.cube(T(70, 20, -60) * Rz(20) * S(20, 20, 40), mat(red));
      sc.cube(T(-70, 40, -60) * Rz(-20) * S(20, 20, 40), mat(green));
      sc.sphere(T(0, 50, -80) * S(20), mat(magenta, 0.8f, 0.995f));
      sc.sphere(T(0, -30, 0) * S(40), mat(yellow, 0.65f, 1, 0, balls ? 0.5f : 0.1f));
      sc.sphere(T(70, 20, 5) * S(20), balls ? mat(red, 0.8f, 0.95f, 0, 0.2f) : mat(red, 0.8f, 0.95f));
      sc.sphere(T(-70, 40, 5) * S(20), mat(green, 0.7f, 0.9f));
      if (balls) sc.quad(T(0, 0, 99) * Rx(180) * S(40, 40, 1), mat(white, 0, 0, 12.0f * li));
      else sc.quad(T(99, -10, -40) * Ry(-90) * S(60, 5, 1), mat(white, 0, 0, 10 * li));
      break;
    }
    case 3:   // scene_menger (key E)
      sc.quad(T(0, 0, -100) * S(9000, 9000, 1), mat(white, 0.8f, 0.999f));
      sponge(sc, T(0, 0, -50) * Rz(15) * S(50), 1, 0.9f, mat(magenta));
      sc.cylinder(T(80, 80, -75) * S(15, 15, 25), mat(blue));
      sc.cylinder(T(-80, 80, -75) * S(15, 15, 25), mat(green));
      sc.cylinder(T(-80, -80, -75) * S(15, 15, 25), mat(red));
      sc.cylinder(T(80, -80, -75) * S(15, 15, 25), mat(yellow));
      sc.sphere(T(80, 80, -30) * S(20), mat(cyan, 0.6f, 0.998f));
      sc.sphere(T(-80, 80, -30) * S(20), mat(green, 0.7f, 0.5f, 0, 0.1f));
      sc.sphere(T(-80, -80, -30) * S(20), mat(red, 0.95f, 0.97f));
      sc.sphere(T(80, -80, -30) * S(20), mat(yellow, 0.5f, 0.999f, 0, 0.25f));
      sc.sphere(T(0, 0, -50) * S(20), mat(white, 1, 1));
      break;
    case 5:   // scene_materials (key T): 11 × 11 spheres, shininess / roughness ramps
      sc.cube(T(0, 0, -50) * S(9000, 9000, 1), mat(white));
      for (int j = -5; j <= 5; j++)
        for (int i = -5; i <= 5; i++)
          sc.sphere(T((float)(30 * i), (float)(30 * j), -41) * S(8),
                    mat(red, (float)(1.0f - 0.075 * (i + 5)), 1.0f - 0.01f * (float)(j + 5)));
      break;
    case 6:   // scene_4boules (key Y) — the north-star scene
      sc.cube(T(0, 0, -51) * S(9000, 9000, 1), mat(white, 0.2f, 0.99999f));
      sc.sphere(T(110, 0, 0) * S(50), mat(magenta, 0.7f, 0.99f, 0, 0.01f));
      sc.sphere(T(-110, 0, 0) * S(50), mat(red, 0.5f, 0.5f, 0, 0.15f));
      sc.sphere(T(0, 110, 0) * S(50), mat(cyan, 0.8f, 0.7f, 0, 0.05f));
      sc.sphere(T(0, -110, 0) * S(50), mat(green, 0.7f, 0.9f, 0, 0.25f));
      sc.quad(T(200, 0, 100) * Ry(-110) * S(20, 20, 1), mat(white, 0, 0, 20 * li));
      break;
    case 7: { // scene_menger_lights (key U)
      sc.cube(T(0, 0, -10) * S(9975, 9975, 1), mat(white, 0.5f, 0.9f));
      sponge(sc, T(0, 0, 42) * Rz(15) * S(50.0f), 1, 0.9f, mat(red));
      const float ring[4][2] = {{-105, 0}, {0, -105}, {0, 105}, {105, 0}};
      const float* ring_col[4] = {blue, cyan, magenta, yellow};
      for (int k = 0; k < 4; ++k) sponge(sc, T(ring[k][0], ring[k][1], 11) * S(20.0f), 0, 0.7f, mat(ring_col[k]));
      sc.sphere(T(-100, -100, 5) * S(15), rgba_mat(1, 1, 1, 0.3f, 0.99f, 0.6f));
      sc.sphere(T(-100, 100, 5) * S(15), rgba_mat(1, 0, 1, 0.2f, 0.8f, 0.4f));
      sc.sphere(T(100, 100, 5) * S(15), rgba_mat(1, 1, 0, 0.4f, 0.6f, 0.2f));
      sc.sphere(T(100, -100, 5) * S(15), rgba_mat(0, 1, 0, 0.1f, 0.4f, 0.1f));
      sc.cube(T(0, 0, 500) * S(1000, 1000, 1), mat(black));
      sc.sphere(T(0, 0, 42) * S(10), mat(white, 0, 0, 10 * li));
      const float lamps[4][2] = {{-105, 0}, {105, 0}, {0, 105}, {0, -105}};
      for (const auto& l : lamps) sc.sphere(T(l[0], l[1], 11) * S(5), mat(white, 0, 0, 10 * li));
      break;
    }
    case 8: { // scene_colonnes (key I): 9 × 9 column capitals
      float ground[4];
      for (int k = 0; k < 4; ++k) ground[k] = 0.6f * white[k] + 0.4f * green[k];
      sc.quad(T(0, 0, -100) * S(90000, 90000, 1), mat(ground, 0.7f, 0.9999f));
      for (int i = -1000; i <= 1000; i += 250)
        for (int j = -1000; j <= 1000; j += 250) {
          const float fi = (float)i, fj = (float)j;
          sc.cylinder(T(fi, fj, -98) * S(60, 60, 2), mat(white));
          sc.cylinder(T(fi, fj, -93) * S(50, 50, 3), mat(white));
          sc.cylinder(T(fi, fj, -85) * S(30, 30, 5), mat(white));
          sc.cylinder(T(fi, fj, 0) * S(20, 20, 80), mat(white));
          sc.cube(T(fi, fj, 90) * S(30, 30, 10), mat(white));
          for (int q = 0; q < 4; ++q)
            sc.cube(T(fi, fj, 105) * Rz(45.0f + 90.0f * q) * T(90, 0, 0) * S(80, 10, 5), mat(white));
          sc.cylinder(T((float)(i + 125), (float)(j + 125), 115) * S(75, 75, 5), mat(white));
          sc.cylinder(T(fi, fj, 115) * S(65, 65, 5), mat(white));
        }
      sc.sphere(T(150, 375, -70) * S(30), mat(yellow, 0.5f, 0.999f));
      sc.sphere(T(100, 125, -70) * S(30), mat(cyan, 0.5f, 0.9f, 0, 0.2f));
      sc.cube(T(125, -125, -80) * Rz(45) * S(20), mat(red, 0.1f, 0.2f));
      break;
    }
    default:
      return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  }
  return sc.finalize();
}

// camera.cpp:53-95 with frame = identity, pivot = origin, radius 145 (montecarlo.cpp:388-389),
// view = modelview · rotateX(-80) (montecarlo.cpp:405), invPV / invV (montecarlo.cpp:439-440)
static void canonical_camera(int W, int H, float* invPV, float* invV) {
  const double fov = 0.78, radius = 145.0;
  const double focal = radius / std::tan(fov / 2.0);
  const double aspect = (double)W / (double)H;
  const double znear = std::max(0.01, focal - radius), zfar = focal + radius;
  const double range_inv = 1.0 / (znear - zfar);
  const double f = 1.0 / std::tan(fov / 2.0);
  Mat4 P;
  std::memset(P.m, 0, sizeof(P.m));
  P(0, 0) = (float)(aspect > 1 ? f / aspect : f);
  P(1, 1) = (float)(aspect > 1 ? f : f * aspect);
  P(2, 2) = (float)((znear + zfar) * range_inv);
  P(2, 3) = (float)(2 * znear * zfar * range_inv);
  P(3, 2) = -1.0f;
  Mat4 MV = Mat4::identity();
  MV(2, 3) = (float)(-focal);
  Mat4 view = MV * Rx(-80);
  Mat4 a = (P * view).inverse(), b = view.inverse();
  std::memcpy(invPV, a.m, 64);
  std::memcpy(invV, b.m, 64);
}

}  // namespace host
}  // namespace mcpt

namespace mcpt {
namespace host {
// Transfo / product entry points of the C ABI (mcpt_image.cpp)
void transfo_translate(float x, float y, float z, float* out) { std::memcpy(out, xf::T(x, y, z).m, 64); }
void transfo_scale(float x, float y, float z, float* out) { std::memcpy(out, xf::S(x, y, z).m, 64); }
void transfo_rotate(int axis, float deg, float* out) {
  const Mat4 r = axis == 0 ? xf::Rx(deg) : (axis == 1 ? xf::Ry(deg) : xf::Rz(deg));
  std::memcpy(out, r.m, 64);
}
void mat4_mul(const float* a, const float* b, float* out) {
  Mat4 A, B;
  std::memcpy(A.m, a, 64);
  std::memcpy(B.m, b, 64);
  const Mat4 r = A * B;
  std::memcpy(out, r.m, 64);
}
}  // namespace host
}  // namespace mcpt

// ======================================================================================
// C ABI — scene half
// ======================================================================================
struct mcpt_scene {
  mcpt::host::PrimScene s;
};

using mcpt::host::Mat4;
using mcpt::host::Material;

static bool unpack(const float* trf16, const float* m7, Mat4& t, Material& m) {
  if (!trf16 || !m7) return false;
  std::memcpy(t.m, trf16, 64);
  std::memcpy(m.rgba, m7, 16);
  m.shininess = m7[4]; m.roughness = m7[5]; m.emissivity = m7[6];
  return true;
}

extern "C" {

int mcpt_scene_create(mcpt_scene** out) {
  if (!out) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *out = new (std::nothrow) mcpt_scene();
  return *out ? MCPT_OK : MCPT_ERR_INVALID_ARG;
}
int mcpt_scene_destroy(mcpt_scene* s) { delete s; return MCPT_OK; }
int mcpt_scene_clear(mcpt_scene* s) { if (!s) return mcpt_err_bare(MCPT_ERR_INVALID_ARG); s->s.clear(); return MCPT_OK; }

#define MCPT_ADD(NAME, METHOD)                                                  \
  int NAME(mcpt_scene* s, const float* trf16, const float* m7) {                \
    Mat4 t; Material m;                                                         \
    if (!s || !unpack(trf16, m7, t, m)) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);            \
    return s->s.METHOD(t, m) >= 0 ? MCPT_OK : MCPT_ERR_INVALID_ARG;             \
  }
MCPT_ADD(mcpt_scene_add_sphere, sphere)
MCPT_ADD(mcpt_scene_add_cube, cube)
MCPT_ADD(mcpt_scene_add_cylinder, cylinder)
MCPT_ADD(mcpt_scene_add_cone, cone)
MCPT_ADD(mcpt_scene_add_oriented_quad, quad)
#undef MCPT_ADD

int mcpt_scene_add_mesh(mcpt_scene* s, const float* vertices, const float* normals, int n_vertices,
                        const unsigned* tri_indices, int n_triangles, const float* bb6, int* mesh_id) {
  if (!s) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  int id = s->s.add_mesh(vertices, normals, n_vertices, tri_indices, n_triangles, bb6);
  if (id < 0) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (mesh_id) *mesh_id = id;
  return MCPT_OK;
}
int mcpt_scene_place_mesh(mcpt_scene* s, int mesh_id, const float* trf16, const float* m7) {
  Mat4 t; Material m;
  if (!s || !unpack(trf16, m7, t, m)) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  return s->s.place_mesh(mesh_id, t, m) >= 0 ? MCPT_OK : MCPT_ERR_INVALID_ARG;
}
int mcpt_scene_mesh_sizes(mcpt_scene* s, int* n_meshes, int* n_nodes, int* n_leaves, int* n_tris, int* n_verts) {
  if (!s || !n_meshes || !n_nodes || !n_leaves || !n_tris || !n_verts) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *n_meshes = (int)s->s.meshes.size();
  *n_nodes = *n_leaves = *n_tris = *n_verts = 0;
  for (const auto& m : s->s.meshes) {
    *n_nodes += (int)(m.nodes.size() / 6);
    *n_leaves += (int)m.leaves.size();
    *n_tris += (int)(m.tris.size() / 3);
    *n_verts += (int)(m.verts.size() / 3);
  }
  return MCPT_OK;
}
int mcpt_scene_get_mesh_buffers(mcpt_scene* s, int* info, float* nodes, int* leaves, int* tris, float* verts,
                                float* normals) {
  if (!s) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  int no = 0, lo = 0, to = 0, vo = 0, k = 0;
  for (const auto& m : s->s.meshes) {
    if (info) { info[4 * k] = no; info[4 * k + 1] = lo; info[4 * k + 2] = m.depth; info[4 * k + 3] = to; }
    if (nodes) std::memcpy(nodes + (size_t)no * 6, m.nodes.data(), m.nodes.size() * 4);
    if (leaves) std::memcpy(leaves + lo, m.leaves.data(), m.leaves.size() * 4);
    if (tris)
      for (size_t i = 0; i < m.tris.size(); ++i) tris[(size_t)to * 3 + i] = (int)m.tris[i] + vo;   // global vertex ids
    if (verts) std::memcpy(verts + (size_t)vo * 3, m.verts.data(), m.verts.size() * 4);
    if (normals) std::memcpy(normals + (size_t)vo * 3, m.normals.data(), m.normals.size() * 4);
    no += (int)(m.nodes.size() / 6); lo += (int)m.leaves.size(); to += (int)(m.tris.size() / 3);
    vo += (int)(m.verts.size() / 3);
    ++k;
  }
  return MCPT_OK;
}

int mcpt_scene_finalize(mcpt_scene* s) { return s ? s->s.finalize() : MCPT_ERR_INVALID_ARG; }
int mcpt_scene_nb_prim(mcpt_scene* s, int* n) { if (!s || !n) return mcpt_err_bare(MCPT_ERR_INVALID_ARG); *n = s->s.count(); return MCPT_OK; }
int mcpt_scene_depth(mcpt_scene* s, int* d) {
  if (!s || !d) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!s->s.finalized) return mcpt_err_bare(MCPT_ERR_NOT_FINALIZED);
  *d = s->s.depth; return MCPT_OK;
}
int mcpt_scene_nb_emissives(mcpt_scene* s, int* n) {
  if (!s || !n) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!s->s.finalized) return mcpt_err_bare(MCPT_ERR_NOT_FINALIZED);
  *n = s->s.nb_emissive; return MCPT_OK;
}
int mcpt_scene_get_buffers(mcpt_scene* s, float* prims, float* nodes, int* leaves) {
  if (!s) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!s->s.finalized) return mcpt_err_bare(MCPT_ERR_NOT_FINALIZED);
  if (prims) std::memcpy(prims, s->s.records.data(), s->s.records.size() * 4);
  if (nodes) std::memcpy(nodes, s->s.nodes.data(), s->s.nodes.size() * 4);
  if (leaves) std::memcpy(leaves, s->s.leaves.data(), s->s.leaves.size() * 4);
  return MCPT_OK;
}
int mcpt_scene_set_material(mcpt_scene* s, int prim, const float* m7) {
  if (!s || !m7 || prim < 0 || prim >= s->s.count()) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!s->s.finalized) return mcpt_err_bare(MCPT_ERR_NOT_FINALIZED);
  float* r = s->s.rec(prim);
  const bool was_emissive = r[58] > 0.0f, is_emissive = m7[6] > 0.0f;
  if (was_emissive != is_emissive) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  std::memcpy(r + 52, m7, 16);
  r[56] = m7[4]; r[57] = m7[5]; r[58] = m7[6];
  return MCPT_OK;
}
int mcpt_scene_build_reference(mcpt_scene* s, int scene_id, float light_intensity) {
  if (!s) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  return mcpt::host::build_reference(s->s, scene_id, light_intensity);
}
int mcpt_camera_canonical(int W, int H, float* invPV16, float* invV16) {
  if (W <= 0 || H <= 0 || !invPV16 || !invV16) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  mcpt::host::canonical_camera(W, H, invPV16, invV16);
  return MCPT_OK;
}

}  // extern "C"
