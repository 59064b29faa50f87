// C++ host API test (include/mcpt.hpp over libmcpt): a caller that builds a scene the way
// montecarlo.cpp does — Transfo products, Material ctors, BVH_GPU_Scene::add_* — gets the
// same buffers, bit for bit, as the library's built-in reference scene.  CPU only unless
// argv[1] == "gpu" (then it also renders through mcpt::Renderer and prints the image sum).
#include <cmath>
#include <cstdio>
#include <cstring>
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
  }
  return fails ? 1 : 0;
}
