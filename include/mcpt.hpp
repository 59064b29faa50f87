// mcpt.hpp — C++ host API over the libmcpt C ABI (include/mcpt.h), header-only.
//
// Mirrors the reference's host interface of the hot path so montecarlo.cpp-style code keeps
// its shape (names and argument meaning of bvh_gpu/scene.h, bvh_gpu/gpu_bvh_scene.h,
// easycppogl/gl_eigen.h):
//
//   GLVec4, GLMat4            Eigen column-major storage (gl_eigen.h:46-60)
//   Transfo::translate/scale/rotateX/rotateY/rotateZ   gl_eigen.cpp:29-105 (degrees)
//   Material (3 ctors + Material::light)               scene.h:30-49
//   PrimData, BB, Mesh/SP_Mesh                         scene.h:15-19, 64-73; mesh.h:85-96
//   ScenePrimitives: clear, nb, add_*, prim_data       scene.h:75-185
//   BVH_GPU_Scene(ScenePrimitives&): clear, add_sphere/add_cube/add_cylinder/add_cone/
//                  add_orientedQuad, add_mesh/place_mesh, finalize, depth(i), nb_prim,
//                  nb_emissives                                  gpu_bvh_scene.h:35-121
//   Renderer: the GL program + accumulation FBO of RTViewer (montecarlo.cpp:384-386, 408-477)
//
// Every matrix product goes through libmcpt (mcpt_mat4_mul) so transforms are bit-identical
// to the reference scenes the library builds.  Errors throw mcpt::Error (the reference has
// no error convention; the C ABI returns status codes).
#ifndef MCPT_HPP_
#define MCPT_HPP_

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mcpt.h"

namespace mcpt {

class Error : public std::runtime_error {
 public:
  Error(const std::string& what, int status)
      : std::runtime_error(what + " failed (" + std::to_string(status) + "): " + mcpt_error_string(status)),
        status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

inline void check(int status, const char* what) {
  if (status != MCPT_OK) throw Error(what, status);
}

struct GLVec4 {
  float v[4];
  GLVec4(float r = 0, float g = 0, float b = 0, float a = 1) : v{r, g, b, a} {}
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};

// column-major 4x4 (Eigen default storage: m[col * 4 + row])
struct GLMat4 {
  float m[16];
  GLMat4() { std::memset(m, 0, sizeof(m)); m[0] = m[5] = m[10] = m[15] = 1.0f; }
  static GLMat4 Identity() { return GLMat4(); }
  float& operator()(int r, int c) { return m[c * 4 + r]; }
  float operator()(int r, int c) const { return m[c * 4 + r]; }
  const float* data() const { return m; }
  GLMat4 operator*(const GLMat4& b) const {
    GLMat4 r;
    check(mcpt_mat4_mul(m, b.m, r.m), "mcpt_mat4_mul");
    return r;
  }
};

namespace Transfo {
inline GLMat4 translate(float x, float y, float z) {
  GLMat4 r;
  check(mcpt_transfo_translate(x, y, z, r.m), "mcpt_transfo_translate");
  return r;
}
inline GLMat4 scale(float sx, float sy, float sz) {
  GLMat4 r;
  check(mcpt_transfo_scale(sx, sy, sz, r.m), "mcpt_transfo_scale");
  return r;
}
inline GLMat4 scale(float s) { return scale(s, s, s); }
inline GLMat4 rotateX(float deg) { GLMat4 r; check(mcpt_transfo_rotate(0, deg, r.m), "rotateX"); return r; }
inline GLMat4 rotateY(float deg) { GLMat4 r; check(mcpt_transfo_rotate(1, deg, r.m), "rotateY"); return r; }
inline GLMat4 rotateZ(float deg) { GLMat4 r; check(mcpt_transfo_rotate(2, deg, r.m), "rotateZ"); return r; }
}  // namespace Transfo

class Material {
 public:
  GLVec4 color_;
  float shininess_, roughness_, emissivity_;
  Material(const GLVec4& color, float shin, float rough, float emi)
      : color_(color), shininess_(shin), roughness_(rough), emissivity_(emi) {}
  Material(const GLVec4& color, float shin, float rough) : Material(color, shin, rough, 0.0f) {}
  explicit Material(const GLVec4& color) : Material(color, 0.0f, 0.0f, 0.0f) {}
  static Material light(const GLVec4& col, float emi) { return Material(col, 0.0f, 0.0f, emi); }
  // the 7 floats the C ABI takes: r, g, b, a(opacity), shininess, roughness, emissivity
  void pack(float out[7]) const {
    for (int k = 0; k < 4; ++k) out[k] = color_[k];
    out[4] = shininess_; out[5] = roughness_; out[6] = emissivity_;
  }
};

struct GLVec3 {
  float v[3];
  GLVec3(float x = 0, float y = 0, float z = 0) : v{x, y, z} {}
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};

// One primitive's record, member for member the reference's PrimData (scene.h:64-73): three
// column-major mat4 (transform, inverse, mesh-BB transform), type (.x type code, .y mesh line),
// colour RGBA (A = opacity), material (shininess, roughness, emissivity, area), padding.
// 16 RGBA32F texels: the tex_prim_ texel layout mcpt_upload_scene takes.
struct PrimData {
  GLMat4 transfo_;
  GLMat4 inv_transfo_;
  GLMat4 inv_mesh_bb_transfo_;
  GLVec4 type_;
  GLVec4 color_;
  GLVec4 mat_info;
  GLVec4 padding2_;
};
static_assert(sizeof(PrimData) == 64 * sizeof(float), "PrimData = 16 RGBA32F texels (scene.h:64-73)");

// BVH node box, the reference's BB (scene.h:15-19: GLVec3 min_, max_): the 2 RGB32F texels of
// tex_bb_ (gpu_bvh_scene.cpp:39-41) mcpt_upload_scene takes per node
struct BB {
  GLVec3 min_;
  GLVec3 max_;
};
static_assert(sizeof(BB) == 6 * sizeof(float), "BB = 2 RGB32F texels (scene.h:15-19)");

// The triangle-mesh data BVH_GPU_Scene::add_mesh reads from the reference's Mesh
// (easycppogl/mesh.h:85-96): positions, normals, triangle vertex indices, bounding box.
class Mesh {
 public:
  std::vector<GLVec3> vertices_;
  std::vector<GLVec3> normals_;
  std::vector<unsigned> tri_indices;
  bool has_bb_ = false;   // false: the vertices' bounding box
  BB bb_;
  int nb_vertices() const { return (int)vertices_.size(); }
  int nb_triangles() const { return (int)(tri_indices.size() / 3); }
};
using SP_Mesh = std::shared_ptr<Mesh>;

// ScenePrimitives (scene.h:75-185): the primitive list.  Owns the library's host scene; the
// records are built by libmcpt (add_prim's inverse and area, prim_bb, sortEmissiveFirst).
class ScenePrimitives {
 public:
  ScenePrimitives() { check(mcpt_scene_create(&s_), "mcpt_scene_create"); }
  ~ScenePrimitives() { mcpt_scene_destroy(s_); }
  ScenePrimitives(const ScenePrimitives&) = delete;
  ScenePrimitives& operator=(const ScenePrimitives&) = delete;

  void clear() { check(mcpt_scene_clear(s_), "mcpt_scene_clear"); }
  int nb() const { int n = 0; check(mcpt_scene_nb_prim(s_, &n), "mcpt_scene_nb_prim"); return n; }
  void add_sphere(const GLMat4& trf, const Material& mat) { add(&mcpt_scene_add_sphere, trf, mat, "add_sphere"); }
  void add_cube(const GLMat4& trf, const Material& mat) { add(&mcpt_scene_add_cube, trf, mat, "add_cube"); }
  void add_cylinder(const GLMat4& trf, const Material& mat) { add(&mcpt_scene_add_cylinder, trf, mat, "add_cylinder"); }
  void add_cone(const GLMat4& trf, const Material& mat) { add(&mcpt_scene_add_cone, trf, mat, "add_cone"); }
  void add_orientedQuad(const GLMat4& trf, const Material& mat) {
    add(&mcpt_scene_add_oriented_quad, trf, mat, "add_orientedQuad");
  }
  // ScenePrimitives::prim_data (scene.h:86-89): the records of a finalized scene, in order
  // (emissive first).  The pointer stays valid until the next prim_data() call.
  const PrimData* prim_data() const {
    const int n = nb(), d = depth_();
    prims_.assign((size_t)n, PrimData());
    std::vector<float> nodes(((size_t(2) << d) - 1) * 6);
    std::vector<int> leaves(size_t(1) << d);
    check(mcpt_scene_get_buffers(s_, reinterpret_cast<float*>(prims_.data()), nodes.data(), leaves.data()),
          "mcpt_scene_get_buffers");
    return prims_.data();
  }
  mcpt_scene* handle() const { return s_; }

 private:
  friend class BVH_GPU_Scene;
  typedef int (*AddFn)(mcpt_scene*, const float*, const float*);
  void add(AddFn fn, const GLMat4& trf, const Material& mat, const char* what) {
    float m7[7];
    mat.pack(m7);
    check(fn(s_, trf.m, m7), what);
  }
  int depth_() const { int d = 0; check(mcpt_scene_depth(s_, &d), "mcpt_scene_depth"); return d; }
  mcpt_scene* s_ = nullptr;
  mutable std::vector<PrimData> prims_;
};

// BVH_GPU_Scene (gpu_bvh_scene.h:35-121) over a caller-owned ScenePrimitives, as in RTViewer
// (montecarlo.cpp:92-93, 133: scene_ declared first, bvh_gpu_scene_(scene_)).  The default
// constructor owns its primitives (a convenience the reference does not have).  finalize()
// = sortEmissiveFirst + BVH_KDtree::init/compute (gpu_bvh_scene.cpp:121-129); the "textures"
// are the flat buffers Renderer::upload sends to the device.
class BVH_GPU_Scene {
 public:
  explicit BVH_GPU_Scene(ScenePrimitives& sc) : scene_(&sc) {}
  BVH_GPU_Scene() : own_(new ScenePrimitives()), scene_(own_.get()) {}
  BVH_GPU_Scene(const BVH_GPU_Scene&) = delete;
  BVH_GPU_Scene& operator=(const BVH_GPU_Scene&) = delete;

  // one of the 8 scenes of montecarlo.cpp:629-795 (keys Q..I = 1..8), finalized
  void build_reference(int scene_id, float light_intensity = 1.2f) {
    check(mcpt_scene_build_reference(s(), scene_id, light_intensity), "mcpt_scene_build_reference");
  }
  void clear() { scene_->clear(); }
  void add_sphere(const GLMat4& trf, const Material& mat) { scene_->add_sphere(trf, mat); }
  void add_cube(const GLMat4& trf, const Material& mat) { scene_->add_cube(trf, mat); }
  void add_cylinder(const GLMat4& trf, const Material& mat) { scene_->add_cylinder(trf, mat); }
  void add_cone(const GLMat4& trf, const Material& mat) { scene_->add_cone(trf, mat); }
  void add_orientedQuad(const GLMat4& trf, const Material& mat) { scene_->add_orientedQuad(trf, mat); }
  // add_mesh (gpu_bvh_scene.cpp:51-74): stores the mesh and builds its own BVH; returns its
  // index for place_mesh (gpu_bvh_scene.h:89-92), which adds an instance with a transform
  int add_mesh(const SP_Mesh& m) {
    // vertex normals are required (Mesh::compute_normals gives them; mesh_inter_geom_info reads them)
    if (!m || m->vertices_.empty() || m->normals_.size() != m->vertices_.size())
      throw Error("add_mesh (mesh needs vertices and one normal per vertex)", MCPT_ERR_INVALID_ARG);
    int id = -1;
    check(mcpt_scene_add_mesh(s(), m->vertices_[0].v, m->normals_[0].v, m->nb_vertices(),
                              m->tri_indices.data(), m->nb_triangles(),
                              m->has_bb_ ? m->bb_.min_.v : nullptr, &id),
          "mcpt_scene_add_mesh");
    return id;
  }
  void place_mesh(int i, const GLMat4& trf, const Material& mat) {
    float m7[7];
    mat.pack(m7);
    check(mcpt_scene_place_mesh(s(), i, trf.m, m7), "mcpt_scene_place_mesh");
  }
  void finalize() { check(mcpt_scene_finalize(s()), "mcpt_scene_finalize"); }
  int depth(int /*bvh*/ = 0) const { return scene_->depth_(); }
  int nb_prim() const { return scene_->nb(); }
  int nb_emissives() const { int n = 0; check(mcpt_scene_nb_emissives(s(), &n), "mcpt_scene_nb_emissives"); return n; }
  int nb_meshes() const {
    int nm = 0, nn = 0, nl = 0, nt = 0, nv = 0;
    check(mcpt_scene_mesh_sizes(s(), &nm, &nn, &nl, &nt, &nv), "mcpt_scene_mesh_sizes");
    return nm;
  }

  // the reference's texture layouts (tex_prim / tex_bb / tex_ind), flattened
  void buffers(std::vector<float>& prims, std::vector<float>& nodes, std::vector<int>& leaves) const {
    const int n = nb_prim(), d = depth();
    prims.assign((size_t)n * 64, 0.0f);
    nodes.assign(((size_t(2) << d) - 1) * 6, 0.0f);
    leaves.assign(size_t(1) << d, 0);
    check(mcpt_scene_get_buffers(s(), prims.data(), nodes.data(), leaves.data()), "mcpt_scene_get_buffers");
  }
  // the root BVH_KDtree's data_BB() / data_ind() (bvh.h:36-44), typed
  void bvh(std::vector<BB>& bbs, std::vector<int>& ind) const {
    std::vector<float> p, n;
    buffers(p, n, ind);
    bbs.resize(n.size() / 6);
    for (size_t i = 0; i < bbs.size(); ++i) {
      bbs[i].min_ = GLVec3(n[i * 6], n[i * 6 + 1], n[i * 6 + 2]);
      bbs[i].max_ = GLVec3(n[i * 6 + 3], n[i * 6 + 4], n[i * 6 + 5]);
    }
  }
  ScenePrimitives& scene() const { return *scene_; }
  mcpt_scene* handle() const { return s(); }

 private:
  mcpt_scene* s() const { return scene_->s_; }
  std::unique_ptr<ScenePrimitives> own_;
  ScenePrimitives* scene_;
};

// canonical camera of RTViewer at aspect W/H: (P·V)^-1 and V^-1, column-major
struct Camera {
  GLMat4 invPV, invV;
  static Camera canonical(int W, int H) {
    Camera c;
    check(mcpt_camera_canonical(W, H, c.invPV.m, c.invV.m), "mcpt_camera_canonical");
    return c;
  }
};

// prg_ray + the RGB32F accumulation FBO (montecarlo.cpp:384-386, 408-477), one GPU
class Renderer {
 public:
  explicit Renderer(int device = 0) { check(mcpt_create(device, &c_), "mcpt_create"); }
  ~Renderer() { mcpt_destroy(c_); }
  Renderer(const Renderer&) = delete;
  Renderer& operator=(const Renderer&) = delete;

  // BVH_GPU_Scene::finalize's texture uploads (gpu_bvh_scene.cpp:121-187): primitives, root
  // BVH and, if the scene has mesh instances, the meshes and their BVHs
  void upload(const BVH_GPU_Scene& sc) {
    std::vector<float> p, n;
    std::vector<int> l;
    sc.buffers(p, n, l);
    check(mcpt_upload_scene(c_, p.data(), sc.nb_prim(), n.data(), l.data(), sc.depth(), sc.nb_emissives()),
          "mcpt_upload_scene");
    int nm = 0, nn = 0, nl = 0, nt = 0, nv = 0;
    check(mcpt_scene_mesh_sizes(sc.handle(), &nm, &nn, &nl, &nt, &nv), "mcpt_scene_mesh_sizes");
    if (nm > 0) {
      std::vector<int> info((size_t)nm * 4), leaves((size_t)nl), tris((size_t)nt * 3);
      std::vector<float> nodes((size_t)nn * 6), verts((size_t)nv * 3), norms((size_t)nv * 3);
      check(mcpt_scene_get_mesh_buffers(sc.handle(), info.data(), nodes.data(), leaves.data(), tris.data(),
                                        verts.data(), norms.data()),
            "mcpt_scene_get_mesh_buffers");
      check(mcpt_upload_meshes(c_, nm, info.data(), nn, nodes.data(), nl, leaves.data(), nt, tris.data(), nv,
                               verts.data(), norms.data()),
            "mcpt_upload_meshes");
    }
  }
  // the reference's own arrays, as BVH_GPU_Scene::finalize hands them to its textures:
  // ScenePrimitives::prim_data() (scene.h:86-89) and the root BVH_KDtree's data_BB() /
  // data_ind() / depth() (bvh.h:24-44) — no repacking on the host
  void upload(const PrimData* prims, int n_prims, const BB* bbs, const int* ind, int depth, int nb_emissives) {
    check(mcpt_upload_scene(c_, reinterpret_cast<const float*>(prims), n_prims, reinterpret_cast<const float*>(bbs),
                            ind, depth, nb_emissives),
          "mcpt_upload_scene");
  }
  void set_target(int W, int H, int band_rows = 8, int world = 1, int rank = 0) {
    check(mcpt_set_target(c_, W, H, band_rows, world, rank), "mcpt_set_target");
    W_ = W; H_ = H;
    check(mcpt_local_rows(c_, &rows_), "mcpt_local_rows");
  }
  // explicit shard: local row i renders global row rows[i]
  void set_target_rows(int W, int H, const std::vector<int>& rows) {
    check(mcpt_set_target_rows(c_, W, H, rows.data(), (int)rows.size()), "mcpt_set_target_rows");
    W_ = W; H_ = H; rows_ = (int)rows.size();
  }
  // this rank's rows of the balanced multi-GPU partition (mcpt_balanced_rows)
  static std::vector<int> balanced_rows(int H, int world, int rank, int band_rows = 8) {
    int n = 0;
    check(mcpt_balanced_rows(H, world, rank, band_rows, nullptr, &n), "mcpt_balanced_rows");
    std::vector<int> rows((size_t)n);
    check(mcpt_balanced_rows(H, world, rank, band_rows, rows.data(), &n), "mcpt_balanced_rows");
    return rows;
  }
  // global row ids of the local rows
  std::vector<int> local_row_ids() const {
    std::vector<int> rows((size_t)rows_);
    if (rows_) check(mcpt_local_row_ids(c_, rows.data()), "mcpt_local_row_ids");
    return rows;
  }
  // numero_pass = first_pass .. first_pass + n_passes - 1, accumulated (blend ONE/ONE)
  void render(const Camera& cam, int first_pass, int n_passes, float date, int bounces, float refract_ind,
              int variant = MCPT_MONTECARLO) {
    check(mcpt_render(c_, cam.invPV.m, cam.invV.m, first_pass, n_passes, date, bounces, refract_ind, variant),
          "mcpt_render");
  }
  void clear_accum() { check(mcpt_clear_accum(c_), "mcpt_clear_accum"); }
  // (local rows × W × 3 sums, pass count)
  int read_accum(std::vector<float>& rgb) const {
    rgb.assign((size_t)rows_ * W_ * 3, 0.0f);
    int n = 0;
    check(mcpt_read_accum(c_, rgb.data(), &n), "mcpt_read_accum");
    return n;
  }
  // the inverse of read_accum (resume): local rows × W × 3 sums holding `passes` passes
  void write_accum(const std::vector<float>& rgb, int passes) {
    if (rgb.size() != (size_t)rows_ * W_ * 3) throw Error("write_accum: wrong size", MCPT_ERR_INVALID_ARG);
    check(mcpt_write_accum(c_, rgb.data(), passes), "mcpt_write_accum");
  }
  // checkpoint / resume of a progressive render (mcpt_checkpoint_save / _load): the file holds
  // the sums, their pass count, the next call's first pass, a tag of the render parameters and
  // the target's identity (H, row ids)
  void save_checkpoint(const std::string& path, int next_pass, const std::string& tag) const {
    check(mcpt_checkpoint_save(c_, path.c_str(), next_pass, tag.c_str()), "mcpt_checkpoint_save");
  }
  // returns the next first pass; throws if the file belongs to another target / shard or its
  // tag differs from this render's
  int load_checkpoint(const std::string& path, const std::string& tag) {
    int next = 0;
    check(mcpt_checkpoint_load(c_, path.c_str(), tag.c_str(), &next), "mcpt_checkpoint_load");
    return next;
  }
  // fs_frag: the averaged image (single-shard target)
  std::vector<float> read_image() const {
    std::vector<float> acc;
    const int n = read_accum(acc);
    std::vector<float> img(acc.size());
    check(mcpt_average(acc.data(), (long long)acc.size(), n > 0 ? n : 1, img.data()), "mcpt_average");
    return img;
  }
  float last_render_ms() const { float ms = 0; check(mcpt_last_render_ms(c_, &ms), "mcpt_last_render_ms"); return ms; }
  // this (full-frame) renderer's accumulator <- the shards' rows (mcpt_gather_rows: peer copies
  // over xGMI inside one process; asynchronous, read_accum / read_image synchronize)
  void gather_rows(const std::vector<const Renderer*>& shards) {
    std::vector<mcpt_ctx*> h;
    for (const Renderer* r : shards) h.push_back(r->c_);
    check(mcpt_gather_rows(c_, h.data(), (int)h.size()), "mcpt_gather_rows");
  }
  void set_traversal(int mode) { check(mcpt_set_traversal(c_, mode), "mcpt_set_traversal"); }
  // render lanes (consecutive launches overlapping each other's tails; same bits): on by default
  void set_render_lanes(bool on) { check(mcpt_set_render_lanes(c_, on ? 1 : 0), "mcpt_set_render_lanes"); }
  // stream schedule knobs (MCPT_TRAVERSAL_STREAM): path slots (0: default), refill threshold (-1: default)
  void set_stream_pool(int slots, int refill) { check(mcpt_set_stream_pool(c_, slots, refill), "mcpt_set_stream_pool"); }
  int width() const { return W_; }
  int height() const { return H_; }
  mcpt_ctx* handle() const { return c_; }

 private:
  mcpt_ctx* c_ = nullptr;
  int W_ = 0, H_ = 0, rows_ = 0;
};

inline void write_pfm(const std::string& path, const std::vector<float>& rgb, int W, int H) {
  check(mcpt_write_pfm(path.c_str(), rgb.data(), W, H), "mcpt_write_pfm");
}
inline void write_png(const std::string& path, const std::vector<float>& rgb, int W, int H) {
  check(mcpt_write_png(path.c_str(), rgb.data(), W, H), "mcpt_write_png");
}

}  // namespace mcpt

#endif  // MCPT_HPP_
