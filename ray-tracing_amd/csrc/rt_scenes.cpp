// rt_scenes.cpp — the src/Scenes.hs scene library, restated over the builder C ABI, plus the two
// benchmark-only scenes of BASELINE.json (config 1 "3-sphere scene", config 5 "100k spheres").
// Every builder consumes the RandGen in the reference's order (mapM/replicateM left to right,
// makeBVH one axis draw per call, makePerlin 768 + 3*255 draws).
#include <cmath>
#include <vector>

#include "rt.h"
#include "rt_internal.h"

namespace {

struct B {
  rt_builder* b;
  int err = 0;
  int chk(int id) {
    if (id < 0 && !err) err = id;
    return id;
  }
  int constant(double r, double g, double bl) { return chk(rt_tex_constant(b, r, g, bl)); }
  int lambertian_c(double r, double g, double bl) { return chk(rt_mat_lambertian(b, constant(r, g, bl))); }
  int sphere(double x, double y, double z, double r, int m) {
    const double c[3] = {x, y, z};
    return chk(rt_obj_sphere(b, c, r, m));
  }
  int rect(int plane, double a0, double a1, double b0, double b1, double k, int m) {
    return chk(rt_obj_rect(b, plane, a0, a1, b0, b1, k, m));
  }
  int cuboid(double x0, double y0, double z0, double x1, double y1, double z1, int m) {
    const double lo[3] = {x0, y0, z0}, hi[3] = {x1, y1, z1};
    return chk(rt_obj_cuboid(b, lo, hi, m));
  }
  int translate(double x, double y, double z, int child) {
    const double o[3] = {x, y, z};
    return chk(rt_obj_translate(b, o, child));
  }
  int bvh(const std::vector<int>& items, double t0 = 0.0, double t1 = 1.0) {
    if (err) return err;
    return chk(rt_obj_bvh(b, items.data(), (int)items.size(), 1, t0, t1));
  }
  double draw() { return b->draw(); }
  double draw_r(double mn, double mx) { return b->draw_r(mn, mx); }
};

enum { XY = 0, XZ = 1, YZ = 2 };

// makeCornellBoxScene (src/Scenes.hs:32-73)
int cornell(B& s, double t0, double t1, int* world, int* lights, double bg[3]) {
  const int red = s.lambertian_c(0.65, 0.05, 0.05);
  const int white = s.lambertian_c(0.73, 0.73, 0.73);
  const int green = s.lambertian_c(0.12, 0.45, 0.15);
  const int light = s.chk(rt_mat_diffuse_light(s.b, s.constant(15, 15, 15)));
  const int light_h = s.rect(XZ, 213, 343, 227, 332, 554, light);
  const int c1 = s.cuboid(0, 0, 0, 165, 330, 165, white);
  const int box1 = s.translate(265, 0, 295, s.chk(rt_obj_rotate(s.b, 1, 15, c1)));
  // `aluminum` and `box2` are let-bound but never used by the reference (lazy, never built).
  const int glass = s.sphere(190, 90, 190, 90, s.chk(rt_mat_dielectric(s.b, 1.5)));
  *world = s.bvh({s.rect(YZ, 0, 555, 0, 555, 555, green), s.rect(YZ, 0, 555, 0, 555, 0, red), light_h,
                  s.rect(XZ, 0, 555, 0, 555, 0, white), s.rect(XZ, 0, 555, 0, 555, 555, white),
                  s.rect(XY, 0, 555, 0, 555, 555, white), box1, glass},
                 t0, t1);
  *lights = s.bvh({light_h, glass}, t0, t1);
  bg[0] = bg[1] = bg[2] = 0.0;
  return s.err;
}

// makeCornellSmokeBoxScene (src/Scenes.hs:75-118)
int cornell_smoke(B& s, double t0, double t1, int* world, int* lights, double bg[3]) {
  const int light = s.chk(rt_mat_diffuse_light(s.b, s.constant(7, 7, 7)));
  const int light_h = s.rect(XZ, 113, 443, 127, 432, 554, light);
  const int red = s.lambertian_c(0.65, 0.05, 0.05);
  const int white = s.lambertian_c(0.73, 0.73, 0.73);
  const int green = s.lambertian_c(0.12, 0.45, 0.15);
  const int b1 = s.translate(265, 0, 295, s.chk(rt_obj_rotate(s.b, 1, 15, s.cuboid(0, 0, 0, 165, 330, 165, white))));
  const int m1 = s.chk(rt_obj_constant_medium(s.b, 0.01, s.constant(0, 0, 0), b1));
  const int b2 = s.translate(130, 0, 65, s.chk(rt_obj_rotate(s.b, 1, -18, s.cuboid(0, 0, 0, 165, 165, 165, white))));
  const int m2 = s.chk(rt_obj_constant_medium(s.b, 0.01, s.constant(1, 1, 1), b2));
  *world = s.bvh({s.rect(YZ, 0, 555, 0, 555, 555, green), s.rect(YZ, 0, 555, 0, 555, 0, red), light_h,
                  s.rect(XZ, 0, 555, 0, 555, 0, white), s.rect(XZ, 0, 555, 0, 555, 555, white),
                  s.rect(XY, 0, 555, 0, 555, 555, white), m1, m2},
                 t0, t1);
  *lights = light_h;
  bg[0] = bg[1] = bg[2] = 0.0;
  return s.err;
}

// makeSimpleLightScene (src/Scenes.hs:133-155)
int simple_light(B& s, double t0, double t1, int* world, int* lights, double bg[3]) {
  const int difflight = s.chk(rt_mat_diffuse_light(s.b, s.constant(4, 4, 4)));
  const int sphere_light = s.sphere(0, 7, 0, 2, difflight);
  const int rect_light = s.rect(XY, 3, 5, 1, 3, -2, difflight);
  const int per = s.chk(rt_tex_perlin(s.b, 1.0));
  const int lam = s.chk(rt_mat_lambertian(s.b, per));
  *world = s.bvh({s.sphere(0, -1000, 0, 1000, lam), s.sphere(0, 2, 0, 2, lam), sphere_light, rect_light}, t0, t1);
  *lights = s.bvh({sphere_light, rect_light}, t0, t1);
  bg[0] = bg[1] = bg[2] = 0.0;
  return s.err;
}

// makeEarthScene (src/Scenes.hs:167-179)
int earth(B& s, double t0, double t1, int earth_tex, int* world, int* lights, double bg[3]) {
  *world = s.bvh({s.sphere(0, 0, 0, 2, s.chk(rt_mat_lambertian(s.b, earth_tex)))}, t0, t1);
  *lights = -1;
  bg[0] = bg[1] = bg[2] = 1.0;
  return s.err;
}

// makeTwoPerlinSpheresScene (src/Scenes.hs:194-211)
int two_perlin(B& s, double t0, double t1, int* world, int* lights, double bg[3]) {
  const int per = s.chk(rt_tex_perlin(s.b, 1.5));
  const int lam = s.chk(rt_mat_lambertian(s.b, per));
  *world = s.bvh({s.sphere(0, -1000, 0, 1000, lam), s.sphere(0, 2, 0, 2, lam)}, t0, t1);
  *lights = -1;
  bg[0] = bg[1] = bg[2] = 0.0;
  return s.err;
}

// makeTwoSpheresScene (src/Scenes.hs:213-237)
int two_spheres(B& s, double t0, double t1, int* world, int* lights, double bg[3]) {
  const int checker = s.chk(rt_tex_checker(s.b, s.constant(0.2, 0.3, 0.1), s.constant(0.9, 0.9, 0.9)));
  const int checker_mat = s.chk(rt_mat_metal(s.b, checker, 0.0));
  const int flat = s.lambertian_c(0.6, 0.2, 0.1);
  *world = s.bvh({s.sphere(0, -10, 0, 10, checker_mat), s.sphere(0, 10, 0, 10, flat)}, t0, t1);
  *lights = -1;
  bg[0] = 0.8; bg[1] = 0.8; bg[2] = 0.9;
  return s.err;
}

// makeRandomSphereM of both random scenes (src/Scenes.hs:284-317 / 364-399); returns -1 for Nothing.
int random_sphere(B& s, int a, int bb, bool moving) {
  const double mat = s.draw();
  const double px = s.draw();
  const double py = s.draw();
  const double cx = (double)a + 0.9 * px, cy = 0.2, cz = (double)bb + 0.9 * py;
  const double dx = cx - 4.0, dy = cy - 0.2, dz = cz - 0.0;
  if (std::sqrt(dx * dx + dy * dy + dz * dz) <= 0.9) return -1;
  if (mat < 0.8) {
    double a1[3], a2[3];
    for (double& v : a1) v = s.draw();  // randomVec3DoubleM
    for (double& v : a2) v = s.draw();
    const int m = s.lambertian_c(a1[0] * a2[0], a1[1] * a2[1], a1[2] * a2[2]);
    if (!moving) return s.sphere(cx, cy, cz, 0.2, m);
    const double mx = s.draw_r(-0.25, 0.25);
    const double mz = s.draw_r(-0.25, 0.25);
    const double c0[3] = {cx, cy, cz}, c1[3] = {cx + mx, cy + 0, cz + mz};
    return s.chk(rt_obj_moving_sphere(s.b, c0, c1, 0.0, 1.0, 0.2, m));
  }
  if (mat < 0.95) {
    double al[3];
    for (double& v : al) v = s.draw_r(0.5, 1.0);  // randomVec3DoubleRM 0.5 1.0
    const double fuzz = s.draw_r(0.0, 0.5);
    return s.sphere(cx, cy, cz, 0.2, s.chk(rt_mat_metal(s.b, s.constant(al[0], al[1], al[2]), fuzz)));
  }
  return s.sphere(cx, cy, cz, 0.2, s.chk(rt_mat_dielectric(s.b, 1.5)));
}

// makeRandomSceneBookOne (src/Scenes.hs:253-317)
int book_one(B& s, int* world, int* lights, double bg[3]) {
  const int ground = s.sphere(0.0, -1000.0, 0.0, 1000, s.lambertian_c(0.5, 0.5, 0.5));
  const int s1 = s.sphere(0.0, 1.0, 0.0, 1.0, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int s2 = s.sphere(-4.0, 1.0, 0.0, 1.0, s.lambertian_c(0.4, 0.2, 0.1));
  const int s3 = s.sphere(4.0, 1.0, 0.0, 1.0, s.chk(rt_mat_metal(s.b, s.constant(0.7, 0.6, 0.5), 0.0)));
  std::vector<int> items = {ground, s1, s2, s3};
  for (int x = -11; x <= 10; ++x)
    for (int y = -11; y <= 10; ++y) {
      const int id = random_sphere(s, x, y, false);
      if (s.err) return s.err;
      if (id >= 0) items.push_back(id);
    }
  *world = s.bvh(items, 0.0, 1.0);
  *lights = -1;
  bg[0] = 0.7; bg[1] = 0.8; bg[2] = 0.9;
  return s.err;
}

// makeRandomScene (src/Scenes.hs:321-399)
int random_scene(B& s, int earth_tex, int* world, int* lights, double bg[3]) {
  const int checker = s.chk(rt_tex_checker(s.b, s.constant(0.2, 0.3, 0.1), s.constant(0.9, 0.9, 0.9)));
  const int ground = s.sphere(0.0, -1000.0, 0.0, 1000, s.chk(rt_mat_lambertian(s.b, checker)));
  const int s1 = s.cuboid(-0.75, 0.0, -0.75, 0.75, 1.5, 0.75, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int s2 = s.sphere(-4.0, 1.0, 0.0, 1.0, s.chk(rt_mat_lambertian(s.b, earth_tex)));
  const int s3 = s.sphere(4.0, 1.0, 0.0, 1.0, s.chk(rt_mat_metal(s.b, s.constant(0.7, 0.6, 0.5), 0.0)));
  std::vector<int> items = {ground, s1, s2, s3};
  for (int x = -11; x <= 10; ++x)
    for (int y = -11; y <= 10; ++y) {
      const int id = random_sphere(s, x, y, true);
      if (s.err) return s.err;
      if (id >= 0) items.push_back(id);
    }
  *world = s.bvh(items, 0.0, 1.0);
  *lights = -1;
  bg[0] = 0.7; bg[1] = 0.8; bg[2] = 0.9;
  return s.err;
}

// makeNextWeekFinalScene (src/Scenes.hs:414-466)
int next_week(B& s, double t0, double t1, int earth_tex, int* world, int* lights, double bg[3]) {
  const int ground = s.lambertian_c(0.48, 0.83, 0.53);
  const int white = s.lambertian_c(0.73, 0.73, 0.73);
  const double w = 100, y0 = 0;
  std::vector<int> boxes1;
  for (int i = 0; i <= 19; ++i)
    for (int j = 0; j <= 19; ++j) {
      const double x0 = (double)i * w - 1000, z0 = (double)j * w - 1000;
      const double x1 = x0 + w;
      const double y1 = s.draw_r(1, 101);
      const double z1 = z0 + w;
      boxes1.push_back(s.cuboid(x0, y0, z0, x1, y1, z1, ground));
    }
  const int b1 = s.bvh(boxes1, 0, 1);
  const int light = s.chk(rt_mat_diffuse_light(s.b, s.constant(7, 7, 7)));
  const int boundary1 = s.sphere(360, 150, 145, 70, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int boundary2 = s.sphere(0, 0, 0, 5000, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int pertext = s.chk(rt_tex_perlin(s.b, 0.1));
  std::vector<int> boxes2;
  for (int i = 0; i < 1000; ++i) {
    double p[3];
    for (double& v : p) v = s.draw_r(0, 165);  // randomVec3DoubleRM 0 165
    boxes2.push_back(s.sphere(p[0], p[1], p[2], 10, white));
  }
  const int b2 = s.bvh(boxes2, 0, 1);
  const double c0[3] = {400, 400, 200}, c1[3] = {430, 400, 200};
  const int ms = s.chk(rt_obj_moving_sphere(s.b, c0, c1, t0, t1, 50, s.lambertian_c(0.7, 0.3, 0.1)));
  const int glass = s.sphere(260, 150, 45, 50, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int metal = s.sphere(0, 150, 145, 50, s.chk(rt_mat_metal(s.b, s.constant(0.8, 0.8, 0.9), 10.0)));
  const int med1 = s.chk(rt_obj_constant_medium(s.b, 0.2, s.constant(0.2, 0.4, 0.9), boundary1));
  const int med2 = s.chk(rt_obj_constant_medium(s.b, 0.0001, s.constant(1, 1, 1), boundary2));
  const int earth_s = s.sphere(400, 200, 400, 100, s.chk(rt_mat_lambertian(s.b, earth_tex)));
  const int per_s = s.sphere(220, 280, 300, 80, s.chk(rt_mat_lambertian(s.b, pertext)));
  const int inst = s.translate(-100, 270, 395, s.chk(rt_obj_rotate(s.b, 1, 15, b2)));
  *world = s.bvh({b1, s.rect(XZ, 113, 443, 127, 432, 554, light), ms, glass, metal, boundary1, med1, med2, earth_s,
                  per_s, inst},
                 t0, t1);
  *lights = -1;
  bg[0] = bg[1] = bg[2] = 0.0;
  return s.err;
}

// Config 1 (BASELINE.json): ground + s1..s3 of makeRandomSceneBookOne (src/Scenes.hs:263-279).
int three_spheres(B& s, int* world, int* lights, double bg[3]) {
  const int ground = s.sphere(0.0, -1000.0, 0.0, 1000, s.lambertian_c(0.5, 0.5, 0.5));
  const int s1 = s.sphere(0.0, 1.0, 0.0, 1.0, s.chk(rt_mat_dielectric(s.b, 1.5)));
  const int s2 = s.sphere(-4.0, 1.0, 0.0, 1.0, s.lambertian_c(0.4, 0.2, 0.1));
  const int s3 = s.sphere(4.0, 1.0, 0.0, 1.0, s.chk(rt_mat_metal(s.b, s.constant(0.7, 0.6, 0.5), 0.0)));
  *world = s.bvh({ground, s1, s2, s3}, 0.0, 1.0);
  *lights = -1;
  bg[0] = 0.7; bg[1] = 0.8; bg[2] = 0.9;
  return s.err;
}

// Config 5 (BASELINE.json / SURVEY.md 8d): n random spheres, radius U(0.05, 0.3), centres
// U([-100,100] x [0.2,5] x [-100,100]), materials drawn as src/Scenes.hs:294-317, + ground.
// Draw order per sphere: mat, cx, cy, cz, r, then the material's draws.
int stress(B& s, int64_t n, int* world, int* lights, double bg[3]) {
  if (n <= 0) n = 100000;
  std::vector<int> items;
  items.reserve((size_t)n + 1);
  items.push_back(s.sphere(0.0, -1000.0, 0.0, 1000, s.lambertian_c(0.5, 0.5, 0.5)));
  for (int64_t i = 0; i < n; ++i) {
    const double mat = s.draw();
    const double cx = s.draw_r(-100, 100), cy = s.draw_r(0.2, 5), cz = s.draw_r(-100, 100);
    const double r = s.draw_r(0.05, 0.3);
    int m;
    if (mat < 0.8) {
      double a1[3], a2[3];
      for (double& v : a1) v = s.draw();
      for (double& v : a2) v = s.draw();
      m = s.lambertian_c(a1[0] * a2[0], a1[1] * a2[1], a1[2] * a2[2]);
    } else if (mat < 0.95) {
      double al[3];
      for (double& v : al) v = s.draw_r(0.5, 1.0);
      const double fuzz = s.draw_r(0.0, 0.5);
      m = s.chk(rt_mat_metal(s.b, s.constant(al[0], al[1], al[2]), fuzz));
    } else {
      m = s.chk(rt_mat_dielectric(s.b, 1.5));
    }
    items.push_back(s.sphere(cx, cy, cz, r, m));
    if (s.err) return s.err;
  }
  *world = s.bvh(items, 0.0, 1.0);
  *lights = -1;
  bg[0] = 0.7; bg[1] = 0.8; bg[2] = 0.9;
  return s.err;
}

}  // namespace

extern "C" int rt_scene_named(rt_builder* b, int id, double t0, double t1, const uint8_t* earth_rgb, int ew, int eh,
                              int64_t param, rt_scene_desc* out) {
  if (!b || !out) {
    rt::set_error("rt_scene_named: null argument");
    return RT_E_INVALID;
  }
  B s{b};
  int world = -1, lights = -1, rc = 0;
  double bg[3] = {0, 0, 0};
  auto earth_tex = [&]() {
    // earthTexture (src/Scenes.hs:157-165): ImageTexture (Just im) w h, or Nothing 0 0
    return s.chk(rt_tex_image(b, earth_rgb, earth_rgb ? ew : 0, earth_rgb ? eh : 0));
  };
  switch (id) {
    case RT_SCENE_CORNELL_BOX: rc = cornell(s, t0, t1, &world, &lights, bg); break;
    case RT_SCENE_CORNELL_SMOKE: rc = cornell_smoke(s, t0, t1, &world, &lights, bg); break;
    case RT_SCENE_SIMPLE_LIGHT: rc = simple_light(s, t0, t1, &world, &lights, bg); break;
    case RT_SCENE_EARTH: rc = earth(s, t0, t1, earth_tex(), &world, &lights, bg); break;
    case RT_SCENE_TWO_PERLIN_SPHERES: rc = two_perlin(s, t0, t1, &world, &lights, bg); break;
    case RT_SCENE_TWO_SPHERES: rc = two_spheres(s, t0, t1, &world, &lights, bg); break;
    case RT_SCENE_RANDOM_BOOK_ONE: rc = book_one(s, &world, &lights, bg); break;
    case RT_SCENE_RANDOM: rc = random_scene(s, earth_tex(), &world, &lights, bg); break;
    case RT_SCENE_NEXT_WEEK_FINAL: rc = next_week(s, t0, t1, earth_tex(), &world, &lights, bg); break;
    case RT_SCENE_THREE_SPHERES: rc = three_spheres(s, &world, &lights, bg); break;
    case RT_SCENE_STRESS_SPHERES: rc = stress(s, param, &world, &lights, bg); break;
    default:
      rt::set_error("rt_scene_named: unknown scene id");
      return RT_E_INVALID;
  }
  if (rc < 0) return rc;
  return rt_builder_finish(b, world, lights, bg, out);
}
