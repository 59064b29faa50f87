// C++ host API test (include/mcpt.hpp over libmcpt): a caller that builds a scene the way
// montecarlo.cpp does — Transfo products, Material ctors, BVH_GPU_Scene::add_* — gets the
// same buffers, bit for bit, as the library's built-in reference scene.  CPU only unless
// argv[1] == "gpu" (then it also renders through mcpt::Renderer and prints the image sum).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "mcpt.hpp"

using mcpt::GLVec4;
using mcpt::Material;
namespace Transfo = mcpt::Transfo;

static GLVec4 OPA(GLVec4 c, float o) { c[3] = o; return c; }
static const GLVec4 BLANC(0.9f, 0.9f, 0.9f, 1), ROUGE(0.9f, 0, 0, 1), VERT(0, 0.9f, 0, 1), CYAN(0, 0.9f, 0.9f, 1),
    MAGENTA(0.9f, 0, 0.9f, 1);

// scene_4boules (montecarlo.cpp:756-770), written against the mirrored API
static void scene_4boules(mcpt::BVH_GPU_Scene& s, float light_intensity) {
  s.add_cube(Transfo::translate(0, 0, -51) * Transfo::scale(9000, 9000, 1), Material(BLANC, 0.2f, 0.99999f));
  s.add_sphere(Transfo::translate(110, 0, 0) * Transfo::scale(50), Material(OPA(MAGENTA, 0.01f), 0.7f, 0.99f));
  s.add_sphere(Transfo::translate(-110, 0, 0) * Transfo::scale(50), Material(OPA(ROUGE, 0.15f), 0.5f, 0.5f));
  s.add_sphere(Transfo::translate(0, 110, 0) * Transfo::scale(50), Material(OPA(CYAN, 0.05f), 0.8f, 0.7f));
  s.add_sphere(Transfo::translate(0, -110, 0) * Transfo::scale(50), Material(OPA(VERT, 0.25f), 0.7f, 0.9f));
  s.add_orientedQuad(Transfo::translate(200, 0, 100) * Transfo::rotateY(-110) * Transfo::scale(20, 20, 1),
                     Material::light(BLANC, 20 * light_intensity));
}

static int same_bits(const void* a, const void* b, size_t n) { return std::memcmp(a, b, n) == 0; }

int main(int argc, char** argv) {
  int fails = 0;
  for (float li : {1.2f, 0.443f}) {
    mcpt::BVH_GPU_Scene mine, ref;
    scene_4boules(mine, li);
    mine.finalize();
    ref.build_reference(6, li);
    std::vector<float> p1, n1, p2, n2;
    std::vector<int> l1, l2;
    mine.buffers(p1, n1, l1);
    ref.buffers(p2, n2, l2);
    const bool ok = mine.nb_prim() == 6 && mine.depth() == 3 && mine.nb_emissives() == 1 && p1.size() == p2.size() &&
                    same_bits(p1.data(), p2.data(), p1.size() * 4) && same_bits(n1.data(), n2.data(), n1.size() * 4) &&
                    l1 == l2;
    std::printf("scene_4boules light %.3f via mcpt.hpp == reference build: %s\n", li, ok ? "ok" : "MISMATCH");
    fails += !ok;
  }
  // clear() + rebuild keeps working (montecarlo.cpp:252: clear before every rebuild)
  {
    mcpt::BVH_GPU_Scene s;
    scene_4boules(s, 1.2f);
    s.finalize();
    s.clear();
    s.add_sphere(Transfo::scale(10), Material(BLANC));
    s.add_sphere(Transfo::translate(30, 0, 0) * Transfo::scale(10), Material::light(BLANC, 5));
    s.finalize();
    const bool ok = s.nb_prim() == 2 && s.depth() == 1 && s.nb_emissives() == 1;
    std::printf("clear + rebuild: %s\n", ok ? "ok" : "FAIL");
    fails += !ok;
  }
  // RTViewer's ownership (montecarlo.cpp:92-93, 133): a ScenePrimitives the caller owns and a
  // BVH_GPU_Scene over it; prim_data() / the root BVH's data_BB / data_ind in the reference's
  // record types carry exactly the flat buffers
  {
    mcpt::ScenePrimitives prims;
    mcpt::BVH_GPU_Scene bvh_scene(prims);
    scene_4boules(bvh_scene, 1.2f);
    bvh_scene.finalize();
    mcpt::BVH_GPU_Scene ref;
    ref.build_reference(6, 1.2f);
    std::vector<float> p2, n2;
    std::vector<int> l2;
    ref.buffers(p2, n2, l2);
    const mcpt::PrimData* pd = prims.prim_data();
    std::vector<mcpt::BB> bbs;
    std::vector<int> ind;
    bvh_scene.bvh(bbs, ind);
    const bool ok = prims.nb() == 6 && &bvh_scene.scene() == &prims &&
                    same_bits(pd, p2.data(), p2.size() * 4) && bbs.size() * 6 == n2.size() &&
                    same_bits(bbs.data(), n2.data(), n2.size() * 4) && ind == l2 &&
                    pd[0].mat_info[2] > 0.0f && pd[0].type_[0] == 5.0f;   // emissive quad first
    std::printf("BVH_GPU_Scene(ScenePrimitives&) + PrimData/BB records == reference build: %s\n", ok ? "ok" : "MISMATCH");
    fails += !ok;
  }
  // add_mesh / place_mesh (gpu_bvh_scene.h:84-92) through mcpt.hpp
  {
    auto m = std::make_shared<mcpt::Mesh>();
    for (int j = 0; j < 3; ++j)
      for (int i = 0; i < 3; ++i) {
        m->vertices_.push_back(mcpt::GLVec3((float)i - 1.0f, (float)j - 1.0f, 0.0f));
        m->normals_.push_back(mcpt::GLVec3(0.0f, 0.0f, 1.0f));
      }
    for (int j = 0; j < 2; ++j)
      for (int i = 0; i < 2; ++i) {
        const unsigned a = (unsigned)(j * 3 + i);
        for (unsigned v : {a, a + 1, a + 3, a + 1, a + 4, a + 3}) m->tri_indices.push_back(v);
      }
    mcpt::ScenePrimitives prims;
    mcpt::BVH_GPU_Scene s(prims);
    const int id = s.add_mesh(m);
    s.place_mesh(id, Transfo::translate(0, 0, 10) * Transfo::scale(30), Material(BLANC, 0.2f, 0.5f));
    s.place_mesh(id, Transfo::translate(60, 0, 10) * Transfo::scale(20), Material(ROUGE));
    s.add_orientedQuad(Transfo::translate(0, 0, 100) * Transfo::scale(20, 20, 1), Material::light(BLANC, 10));
    s.finalize();
    bool threw = false;
    try {
      auto bad = std::make_shared<mcpt::Mesh>();
      bad->vertices_ = m->vertices_;   // no normals
      bad->tri_indices = m->tri_indices;
      s.add_mesh(bad);
    } catch (const mcpt::Error&) {
      threw = true;
    }
    const bool ok = id == 0 && s.nb_meshes() == 1 && s.nb_prim() == 3 && s.nb_emissives() == 1 && threw;
    std::printf("add_mesh + place_mesh: %s\n", ok ? "ok" : "FAIL");
    fails += !ok;
  }
  // errors surface as mcpt::Error with the C status
  try {
    mcpt::BVH_GPU_Scene s;
    s.build_reference(99);
    std::printf("bad scene id: FAIL (no throw)\n");
    ++fails;
  } catch (const mcpt::Error& e) {
    std::printf("bad scene id throws: ok (%d)\n", e.status());
  }
  if (argc > 1 && std::strcmp(argv[1], "gpu") == 0) {
    mcpt::BVH_GPU_Scene s;
    s.build_reference(6);
    mcpt::Renderer r(0);
    r.upload(s);
    r.set_target(64, 48);
    r.render(mcpt::Camera::canonical(64, 48), 1, 4, 0.0f, 8, 1.0f);
    std::vector<float> img = r.read_image();
    double sum = 0;
    for (float v : img) sum += v;
    std::printf("gpu image sum %.6f\n", sum);
    fails += !(std::isfinite(sum) && sum > 0);
    // the reference's own arrays passed straight through (INTEGRATION.md adapter):
    // ScenePrimitives::prim_data() + BVH_KDtree::data_BB()/data_ind()/depth()
    std::vector<float> acc1, acc2;
    const int n1 = r.read_accum(acc1);
    mcpt::ScenePrimitives prims;
    mcpt::BVH_GPU_Scene s2(prims);
    scene_4boules(s2, 1.2f);
    s2.finalize();
    std::vector<mcpt::BB> bbs;
    std::vector<int> ind;
    s2.bvh(bbs, ind);
    std::vector<mcpt::PrimData> pd(prims.prim_data(), prims.prim_data() + prims.nb());
    mcpt::Renderer r2(0);
    r2.upload(pd.data(), (int)pd.size(), bbs.data(), ind.data(), s2.depth(), s2.nb_emissives());
    r2.set_target(64, 48);
    r2.render(mcpt::Camera::canonical(64, 48), 1, 4, 0.0f, 8, 1.0f);
    const int n2 = r2.read_accum(acc2);
    const bool same = n1 == n2 && acc1.size() == acc2.size() && same_bits(acc1.data(), acc2.data(), acc1.size() * 4);
    std::printf("gpu reference-layout upload bit-equal: %s\n", same ? "ok" : "MISMATCH");
    fails += !same;
  }
  return fails ? 1 : 0;
}
