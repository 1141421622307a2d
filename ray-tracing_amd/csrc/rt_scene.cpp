// rt_scene.cpp — host-side scene construction behind the C ABI (include/rt.h).
//
// Mirrors the reference's construction API (src/Lib.hs constructors, makeBVH, makePerlin,
// newCamera) and the src/Scenes.hs builders, writing straight into the flat record arrays the
// device consumes (rt_node / rt_material / rt_texture / rt_perlin). Haskell value sharing
// (the Cornell light in both trees, `BVHNode h h`, a medium's boundary) becomes id sharing.
// The RandGen threaded through construction is a SplitMix64 (seed, gamma) pair consumed in the
// reference's order, so the generator handed back (`g1`, app/Main.hs:41,49) matches.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt.h"
#include "rt_internal.h"

namespace {

constexpr double kEps = 0.0001;               // src/Lib.hs:76-77
constexpr double kPi = 3.141592653589793;     // GHC pi
constexpr double kInf = INFINITY;

inline double gmax(double x, double y) { return x <= y ? y : x; }  // GHC Ord default
inline double gmin(double x, double y) { return x <= y ? x : y; }

using rt::Box;
}  // namespace



namespace {

thread_local std::string g_err;

int fail(const char* msg) {
  g_err = msg;
  return RT_E_INVALID;
}

int push_node(rt_builder* b, int type, const double* f, int nf, int a, int bb, int c) {
  rt_node n;
  std::memset(&n, 0, sizeof n);
  n.type = type;
  for (int i = 0; i < nf; ++i) n.f[i] = f[i];
  n.a = a;
  n.b = bb;
  n.c = c;
  b->nodes.push_back(n);
  return (int)b->nodes.size() - 1;
}

bool valid_node(const rt_builder* b, int id) { return id >= 0 && id < (int)b->nodes.size() && b->nodes[id].type != RT_NODE_EXT; }
bool valid_mat(const rt_builder* b, int id) { return id >= 0 && id < (int)b->materials.size(); }
bool valid_tex(const rt_builder* b, int id) { return id >= 0 && id < (int)b->textures.size(); }

// boundingBox (src/Lib.hs:905-927); returns false for Unhittable (the reference errors).
bool bounding_box(const rt_builder* b, int id, Box* out) {
  const rt_node& n = b->nodes[id];
  switch (n.type) {
    case RT_NODE_SPHERE:
      for (int i = 0; i < 3; ++i) { out->mn[i] = n.f[i] - n.f[3]; out->mx[i] = n.f[i] + n.f[3]; }
      return true;
    case RT_NODE_MOVING_SPHERE: {
      const double r = b->nodes[id + 1].f[3];
      Box b0, b1;
      for (int i = 0; i < 3; ++i) {
        b0.mn[i] = n.f[i] - r; b0.mx[i] = n.f[i] + r;
        b1.mn[i] = n.f[3 + i] - r; b1.mx[i] = n.f[3 + i] + r;
      }
      for (int i = 0; i < 3; ++i) { out->mn[i] = gmin(b0.mn[i], b1.mn[i]); out->mx[i] = gmax(b0.mx[i], b1.mx[i]); }
      return true;
    }
    case RT_NODE_RECT_XY:
      out->mn[0] = n.f[0]; out->mn[1] = n.f[2]; out->mn[2] = n.f[4] - kEps;
      out->mx[0] = n.f[1]; out->mx[1] = n.f[3]; out->mx[2] = n.f[4] + kEps;
      return true;
    case RT_NODE_RECT_XZ:
      out->mn[0] = n.f[0]; out->mn[1] = n.f[4] - kEps; out->mn[2] = n.f[2];
      out->mx[0] = n.f[1]; out->mx[1] = n.f[4] + kEps; out->mx[2] = n.f[3];
      return true;
    case RT_NODE_RECT_YZ:
      out->mn[0] = n.f[4] - kEps; out->mn[1] = n.f[0]; out->mn[2] = n.f[2];
      out->mx[0] = n.f[4] + kEps; out->mx[1] = n.f[1]; out->mx[2] = n.f[3];
      return true;
    case RT_NODE_BVH:
    case RT_NODE_CUBOID:
      for (int i = 0; i < 3; ++i) { out->mn[i] = n.f[i]; out->mx[i] = n.f[3 + i]; }
      return true;
    case RT_NODE_TRANSLATE: {
      Box c;
      if (!bounding_box(b, n.a, &c)) return false;
      for (int i = 0; i < 3; ++i) { out->mn[i] = c.mn[i] + n.f[i]; out->mx[i] = c.mx[i] + n.f[i]; }
      return true;
    }
    case RT_NODE_ROTATE:
      *out = b->rotate_boxes.at(id);
      return true;
    case RT_NODE_CONSTANT_MEDIUM:
      return bounding_box(b, n.a, out);
    default:
      return false;
  }
}

// rotatePoint (src/Lib.hs:763-774)
void rotate_point(int axis, double s, double c, const double p[3], double o[3]) {
  if (axis == 0) { o[0] = p[0]; o[1] = c * p[1] - s * p[2]; o[2] = s * p[1] + c * p[2]; }
  else if (axis == 1) { o[0] = c * p[0] + s * p[2]; o[1] = p[1]; o[2] = -s * p[0] + c * p[2]; }
  else { o[0] = c * p[0] - s * p[1]; o[1] = s * p[0] + c * p[1]; o[2] = p[2]; }
}

int node_size(const rt_builder* b, int id) { return b->nodes[id].c; }

// makeBVH (src/Lib.hs:941-961)
int make_bvh(rt_builder* b, std::vector<int> items) {
  const double rd = b->draw_r(0.0, 3.0);
  const double fa = std::floor(rd);
  if (!(fa >= 0.0 && fa < 3.0)) return fail("makeBVH: axis index out of range (draw = 1.0, `!!` would fail)");
  const int axis = (int)fa;
  const int n = (int)items.size();
  std::vector<Box> boxes(n);
  for (int i = 0; i < n; ++i)
    if (!bounding_box(b, items[i], &boxes[i])) return fail("makeBVH: cannot bound an Unhittable");
  // boxCompare: compare on box_min of the chosen axis (src/Lib.hs:963-968); LT iff x < y.
  auto lt = [&](int i, int j) { return boxes[i].mn[axis] < boxes[j].mn[axis]; };
  int left, right;
  if (n == 1) {
    left = right = items[0];
  } else if (n == 2) {
    if (lt(0, 1)) { left = items[0]; right = items[1]; }
    else { left = items[1]; right = items[0]; }
  } else {
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), lt);  // Data.Sequence.sortBy is stable
    const int half = n / 2;
    std::vector<int> l(half), r(n - half);
    for (int i = 0; i < half; ++i) l[i] = items[order[i]];
    for (int i = half; i < n; ++i) r[i - half] = items[order[i]];
    left = make_bvh(b, l);
    if (left < 0) return left;
    right = make_bvh(b, r);
    if (right < 0) return right;
  }
  Box bl, br;
  if (!bounding_box(b, left, &bl) || !bounding_box(b, right, &br)) return fail("makeBVH: cannot bound child");
  double f[6];
  for (int i = 0; i < 3; ++i) { f[i] = gmin(bl.mn[i], br.mn[i]); f[3 + i] = gmax(bl.mx[i], br.mx[i]); }
  return push_node(b, RT_NODE_BVH, f, 6, left, right, n);
}

}  // namespace

namespace rt {
void set_error(const std::string& s) { g_err = s; }
const char* last_error() { return g_err.c_str(); }
}  // namespace rt

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_err.c_str(); }

void rt_rand_gen(int64_t s, uint64_t out_gen[2]) { rt::mk_smgen((uint64_t)s, out_gen); }

double rt_random_double(uint64_t gen[2]) { return rt::word_to_draw(rt::sm_next(gen[0], gen[1])); }

int rt_builder_create(const uint64_t gen[2], rt_builder** out) {
  if (!gen || !out) return fail("rt_builder_create: null argument");
  rt_builder* b = new (std::nothrow) rt_builder();
  if (!b) return RT_E_NOMEM;
  b->seed = gen[0];
  b->gamma = gen[1];
  *out = b;
  return RT_OK;
}

void rt_builder_destroy(rt_builder* b) { delete b; }

void rt_builder_gen(const rt_builder* b, uint64_t out_gen[2]) {
  out_gen[0] = b->seed;
  out_gen[1] = b->gamma;
}

int rt_tex_constant(rt_builder* b, double r, double g, double bl) {
  rt_texture t;
  std::memset(&t, 0, sizeof t);
  t.type = RT_TEX_CONSTANT;
  t.f[0] = r; t.f[1] = g; t.f[2] = bl;
  b->textures.push_back(t);
  return (int)b->textures.size() - 1;
}

int rt_tex_checker(rt_builder* b, int odd_tex, int even_tex) {
  if (!valid_tex(b, odd_tex) || !valid_tex(b, even_tex)) return fail("rt_tex_checker: bad texture id");
  rt_texture t;
  std::memset(&t, 0, sizeof t);
  t.type = RT_TEX_CHECKER;
  t.a = odd_tex;
  t.b = even_tex;
  b->textures.push_back(t);
  return (int)b->textures.size() - 1;
}

// makePerlin (src/Lib.hs:424-439)
int rt_tex_perlin(rt_builder* b, double scale) {
  rt_perlin p;
  for (int i = 0; i < 256; ++i)
    for (int k = 0; k < 3; ++k) p.ranvec[i][k] = b->draw_r(-1.0, 1.0);  // randomVec3DoubleRM (-1) 1
  int32_t* perms[3] = {p.perm_x, p.perm_y, p.perm_z};
  for (int q = 0; q < 3; ++q) {  // perlinGeneratePerm
    int32_t* a = perms[q];
    for (int i = 0; i < 256; ++i) a[i] = i;
    for (int i = 255; i >= 1; --i) {
      const int target = (int)std::floor(b->draw_r(0.0, (double)i));  // randomIntRM 0 i
      std::swap(a[i], a[target]);
    }
  }
  b->perlins.push_back(p);
  rt_texture t;
  std::memset(&t, 0, sizeof t);
  t.type = RT_TEX_PERLIN;
  t.a = (int)b->perlins.size() - 1;
  t.f[0] = scale;
  b->textures.push_back(t);
  return (int)b->textures.size() - 1;
}

int rt_tex_image(rt_builder* b, const uint8_t* rgb, int width, int height) {
  rt_texture t;
  std::memset(&t, 0, sizeof t);
  t.type = RT_TEX_IMAGE;
  if (!rgb) {  // ImageTexture Nothing 0 0 (earthTexture's Left branch, src/Scenes.hs:161)
    t.a = -1;
    t.b = width;
    t.c = height;
  } else {
    if (width <= 0 || height <= 0) return fail("rt_tex_image: bad size");
    rt_image im;
    im.offset = (int64_t)b->pool.size();
    im.width = width;
    im.height = height;
    b->pool.insert(b->pool.end(), rgb, rgb + (size_t)width * height * 3);
    b->images.push_back(im);
    t.a = (int)b->images.size() - 1;
    t.b = width;
    t.c = height;
  }
  b->textures.push_back(t);
  return (int)b->textures.size() - 1;
}

static int push_mat(rt_builder* b, int type, int tex, double param) {
  if (type != RT_MAT_DIELECTRIC && !valid_tex(b, tex)) return fail("material: bad texture id");
  rt_material m;
  std::memset(&m, 0, sizeof m);
  m.type = type;
  m.texture = type == RT_MAT_DIELECTRIC ? -1 : tex;
  m.param = param;
  b->materials.push_back(m);
  return (int)b->materials.size() - 1;
}
int rt_mat_lambertian(rt_builder* b, int tex) { return push_mat(b, RT_MAT_LAMBERTIAN, tex, 0.0); }
int rt_mat_metal(rt_builder* b, int tex, double fuzz) { return push_mat(b, RT_MAT_METAL, tex, fuzz); }
int rt_mat_dielectric(rt_builder* b, double ref_idx) { return push_mat(b, RT_MAT_DIELECTRIC, -1, ref_idx); }
int rt_mat_diffuse_light(rt_builder* b, int tex) { return push_mat(b, RT_MAT_DIFFUSE_LIGHT, tex, 0.0); }
int rt_mat_isotropic(rt_builder* b, int tex) { return push_mat(b, RT_MAT_ISOTROPIC, tex, 0.0); }

int rt_obj_sphere(rt_builder* b, const double c[3], double r, int mat) {
  if (!valid_mat(b, mat)) return fail("sphere: bad material id");
  const double f[4] = {c[0], c[1], c[2], r};
  return push_node(b, RT_NODE_SPHERE, f, 4, mat, 0, 1);
}

// movingSphere c0 c1 t0 t1 = MovingSphere c0 c1 t0 t1 (t1 - t0)  (src/Lib.hs:590-592)
int rt_obj_moving_sphere(rt_builder* b, const double c0[3], const double c1[3], double t0, double t1, double r,
                         int mat) {
  if (!valid_mat(b, mat)) return fail("movingSphere: bad material id");
  const double f[6] = {c0[0], c0[1], c0[2], c1[0], c1[1], c1[2]};
  const int id = push_node(b, RT_NODE_MOVING_SPHERE, f, 6, mat, 0, 1);
  const double e[4] = {t0, t1, t1 - t0, r};
  push_node(b, RT_NODE_EXT, e, 4, 0, 0, 0);
  return id;
}

int rt_obj_rect(rt_builder* b, int plane, double a0, double a1, double b0, double b1, double k, int mat) {
  if (plane < 0 || plane > 2) return fail("rect: plane must be 0 (XY), 1 (XZ) or 2 (YZ)");
  if (!valid_mat(b, mat)) return fail("rect: bad material id");
  const double f[5] = {a0, a1, b0, b1, k};
  return push_node(b, RT_NODE_RECT_XY + plane, f, 5, mat, 0, 1);
}

int rt_obj_cuboid(rt_builder* b, const double pmin[3], const double pmax[3], int mat) {
  if (!valid_mat(b, mat)) return fail("cuboid: bad material id");
  const double f[6] = {pmin[0], pmin[1], pmin[2], pmax[0], pmax[1], pmax[2]};
  return push_node(b, RT_NODE_CUBOID, f, 6, mat, 0, 1);
}

int rt_obj_translate(rt_builder* b, const double off[3], int child) {
  if (!valid_node(b, child)) return fail("translate: bad child id");
  return push_node(b, RT_NODE_TRANSLATE, off, 3, child, 0, node_size(b, child));
}

// rotate (src/Lib.hs:732-761), including its 3x3x3 corner fold (i,j,k in {0,1,2}).
int rt_obj_rotate(rt_builder* b, int axis, double angle, int child) {
  if (axis < 0 || axis > 2) return fail("rotate: axis must be 0, 1 or 2");
  if (!valid_node(b, child)) return fail("rotate: bad child id");
  const double rad = angle * kPi / 180.0;
  const double s = std::sin(rad), c = std::cos(rad);
  Box hb;
  if (!bounding_box(b, child, &hb)) return fail("rotate: cannot bound an Unhittable");
  double mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
  // foldr over [(i,j,k) | i <- [0,1,2], j <- [0,1,2], k <- [0,1,2]]: last element first.
  for (int idx = 26; idx >= 0; --idx) {
    const double i = idx / 9, j = (idx / 3) % 3, k = idx % 3;
    const double p[3] = {i * hb.mx[0] + (1 - i) * hb.mn[0], j * hb.mx[1] + (1 - j) * hb.mn[1],
                         k * hb.mx[2] + (1 - k) * hb.mn[2]};
    double q[3];
    rotate_point(axis, s, c, p, q);
    for (int a = 0; a < 3; ++a) { mn[a] = gmin(q[a], mn[a]); mx[a] = gmax(q[a], mx[a]); }
  }
  const double f[2] = {s, c};
  const int id = push_node(b, RT_NODE_ROTATE, f, 2, child, axis, node_size(b, child));
  Box rb;
  for (int a = 0; a < 3; ++a) { rb.mn[a] = mn[a]; rb.mx[a] = mx[a]; }
  b->rotate_boxes[id] = rb;
  return id;
}

// constantMedium density tex = ConstantMedium (-1 / density) (Isotropic tex)  (src/Lib.hs:789-791)
int rt_obj_constant_medium(rt_builder* b, double density, int tex, int boundary) {
  if (!valid_node(b, boundary)) return fail("constantMedium: bad boundary id");
  const int mat = rt_mat_isotropic(b, tex);
  if (mat < 0) return mat;
  const double f[1] = {-1 / density};
  return push_node(b, RT_NODE_CONSTANT_MEDIUM, f, 1, boundary, mat, 1);
}

int rt_obj_unhittable(rt_builder* b) { return push_node(b, RT_NODE_UNHITTABLE, nullptr, 0, 0, 0, 0); }

int rt_obj_bvh(rt_builder* b, const int* items, int n, int has_time, double t0, double t1) {
  (void)has_time; (void)t0; (void)t1;  // mtime only threads through boundingBox unused (Lib.hs:905-927)
  if (!items || n <= 0) return fail("makeBVH: empty sequence (the reference pattern-match fails)");
  std::vector<int> v(items, items + n);
  for (int id : v)
    if (!valid_node(b, id)) return fail("makeBVH: bad item id");
  return make_bvh(b, v);
}

int rt_builder_finish(rt_builder* b, int world, int lights, const double bg[3], rt_scene_desc* d) {
  if (!valid_node(b, world)) return fail("finish: bad world id");
  if (lights >= 0 && !valid_node(b, lights)) return fail("finish: bad lights id");
  if (lights >= 0 && b->nodes[lights].type == RT_NODE_UNHITTABLE) lights = -1;
  std::memset(d, 0, sizeof *d);
  d->nodes = b->nodes.data();
  d->n_nodes = (int)b->nodes.size();
  d->world_root = world;
  d->lights_root = lights;
  d->materials = b->materials.data();
  d->n_materials = (int)b->materials.size();
  d->textures = b->textures.data();
  d->n_textures = (int)b->textures.size();
  d->perlins = b->perlins.data();
  d->n_perlins = (int)b->perlins.size();
  d->images = b->images.data();
  d->n_images = (int)b->images.size();
  d->image_pool = b->pool.data();
  d->image_pool_bytes = (int64_t)b->pool.size();
  for (int i = 0; i < 3; ++i) d->background[i] = bg[i];
  return RT_OK;
}

// ------------------------------------------------------------------ cameras
// newCamera (src/Lib.hs:1280-1295)
void rt_camera_new(const double lf[3], const double la[3], const double vup[3], double vfov, double aspect,
                   double aperture, double focus, double t0, double t1, rt_camera* o) {
  auto sub = [](const double* a, const double* b, double* r) { for (int i = 0; i < 3; ++i) r[i] = a[i] - b[i]; };
  auto unit = [](double* v) {
    const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int i = 0; i < 3; ++i) v[i] = v[i] / l;
  };
  auto cross = [](const double* a, const double* b, double* r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
  };
  const double lens_radius = aperture / 2.0;
  const double theta = vfov * kPi / 180.0;
  const double half_height = std::tan(theta / 2.0);
  const double half_width = aspect * half_height;
  double w[3], u[3], v[3];
  sub(lf, la, w);
  unit(w);
  cross(vup, w, u);
  unit(u);
  cross(w, u, v);
  for (int i = 0; i < 3; ++i) {
    o->origin[i] = lf[i];
    o->llc[i] = ((lf[i] - u[i] * (half_width * focus)) - v[i] * (half_height * focus)) - w[i] * focus;
    o->horiz[i] = u[i] * (2 * half_width * focus);
    o->vert[i] = v[i] * (2 * half_height * focus);
    o->u[i] = u[i];
    o->v[i] = v[i];
    o->w[i] = w[i];
  }
  o->lens_radius = lens_radius;
  o->t0 = t0;
  o->t1 = t1;
}

int rt_camera_named(int id, int width, int height, rt_camera* out) {
  if (width <= 0 || height <= 0 || !out) return fail("rt_camera_named: bad size");
  const double aspect = (double)width / (double)height;
  const double up[3] = {0.0, 1.0, 0.0};
  switch (id) {
    case RT_CAM_CORNELL: {  // src/Scenes.hs:120-131
      const double lf[3] = {278, 278, -800}, la[3] = {278, 278, 0.0};
      rt_camera_new(lf, la, up, 40.0, aspect, 0.0, 10.0, 0.0, 1.0, out);
      return RT_OK;
    }
    case RT_CAM_TWO_SPHERES: {  // src/Scenes.hs:181-192
      const double lf[3] = {26.0, 4.0, 6.0}, la[3] = {0.0, 2.0, 0.0};
      rt_camera_new(lf, la, up, 20.0, aspect, 0.1, 20.0, 0.0, 1.0, out);
      return RT_OK;
    }
    case RT_CAM_RANDOM_SCENE: {  // src/Scenes.hs:239-250
      const double lf[3] = {13.0, 2.0, 3.0}, la[3] = {0.0, 0.0, 0.0};
      rt_camera_new(lf, la, up, 20.0, aspect, 0.1, 10.0, 0.0, 1.0, out);
      return RT_OK;
    }
    case RT_CAM_NEXT_WEEK: {  // src/Scenes.hs:401-412
      const double lf[3] = {575, 278, -525}, la[3] = {320, 278, 0.0};
      rt_camera_new(lf, la, up, 40.0, aspect, 0.1, 580.0, 0.0, 1.0, out);
      return RT_OK;
    }
  }
  return fail("rt_camera_named: unknown camera id");
}

// ------------------------------------------------------------------ PPM
// P3 header (app/Main.hs:59-61) and printRow/showRow (src/Lib.hs:299-305): one line per row,
// "r g b r g b ..." joined by single spaces.
int rt_write_ppm(const uint8_t* rgb, int width, int height, char* buf, size_t cap, size_t* out_len) {
  if (!rgb || width <= 0 || height <= 0) return fail("rt_write_ppm: bad arguments");
  std::string s;
  s.reserve((size_t)width * height * 12 + 32);
  s += "P3\n";
  s += std::to_string(width) + " " + std::to_string(height) + "\n255\n";
  char tmp[8];
  for (int row = 0; row < height; ++row) {
    for (int x = 0; x < width; ++x) {
      for (int c = 0; c < 3; ++c) {
        const int n = std::snprintf(tmp, sizeof tmp, "%u", (unsigned)rgb[((size_t)row * width + x) * 3 + c]);
        if (x || c) s += ' ';
        s.append(tmp, (size_t)n);
      }
    }
    s += '\n';
  }
  if (out_len) *out_len = s.size();
  if (buf && cap) std::memcpy(buf, s.data(), std::min(cap, s.size()));
  return RT_OK;
}

// ------------------------------------------------------------------ float dump
// The per-pixel averages before albedoToColor (rt_render's out_linear), for the per-channel tolerance
// metric. PFM: "PF\n<W> <H>\n-1.0\n" then little-endian float32 RGB rows from the BOTTOM row up (the
// format's order). `f64` != 0 writes the same layout with doubles under the header "PF64" (no
// rounding: the dump parity tests compare). NaN pixels (the reference prints them as 0) stay NaN.
int rt_write_pfm(const double* linear, int width, int height, int f64, char* buf, size_t cap, size_t* out_len) {
  if (!linear || width <= 0 || height <= 0) return fail("rt_write_pfm: bad arguments");
  const std::string head = std::string(f64 ? "PF64" : "PF") + "\n" + std::to_string(width) + " " +
                           std::to_string(height) + "\n-1.0\n";
  const size_t px = (size_t)width * height * 3, elem = f64 ? sizeof(double) : sizeof(float);
  const size_t n = head.size() + px * elem;
  if (out_len) *out_len = n;
  if (!buf || !cap) return RT_OK;
  std::string s;
  s.reserve(n);
  s += head;
  for (int row = height - 1; row >= 0; --row) {
    const double* src = linear + (size_t)row * width * 3;
    for (int i = 0; i < width * 3; ++i) {
      unsigned char b[8];
      if (f64) {
        std::memcpy(b, &src[i], 8);
      } else {
        const float f = (float)src[i];
        std::memcpy(b, &f, 4);
      }
      s.append((const char*)b, elem);  // (x86-64 / gfx950 hosts are little-endian)
    }
  }
  std::memcpy(buf, s.data(), std::min(cap, s.size()));
  return RT_OK;
}

}  // extern "C"
