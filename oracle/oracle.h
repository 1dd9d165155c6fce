/* ORACLE — test infrastructure only.
 *
 * CPU restatement (f64, scalar C++) of lumo's render hot path, used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker / baseline.
 * The product (lumo_amd) never links, loads or calls anything under oracle/.
 *
 * It consumes the same flattened scene and camera (include/lumo_amd.h) the GPU path
 * consumes, and restates, function by function, with file:line citations in oracle.cpp:
 *   renderer.rs / renderer/task.rs   tile tasks, per-pixel samplers, adaptive-RR delta
 *   samplers.rs, rng.rs, rng/maps.rs  MultiJittered sampler, Xorshiftr128+, disk maps
 *   integrator.rs, path_trace.rs      path tracing with NEE + MIS + Russian roulette
 *   scene.rs, object/{bvh,kdtree,triangle,rectangle,aabb}.rs  traversal + intersection
 *   hit.rs, ray.rs, onb.rs, efloat.rs robust spawning, shading frame
 *   material.rs, bsdf.rs, bxdf.rs, bxdf/{scatter,microfacet}.rs, microfacet.rs
 *                                    Lambertian, MfDiffuse, MfConductor, MfDielectric, Light
 *   color/{color,wavelength,spectrum,dense_spectrum,xyz,space}.rs  hero wavelengths
 *   camera.rs, film.rs, film/tile.rs, filter.rs, tone_mapping.rs
 *
 * Parity pins: lumo's Rust crate cannot be built here (no cargo; srgb.coeff missing), so
 * the oracle is pinned by the reference's own known-answer vectors (spectrum_tests.rs)
 * and property tests (kd-tree reachability, hit/hit_t consistency, scene visibility,
 * filter integrals) — see tests/ and DESIGN.md §Oracle.
 *
 * Two sample-stream orders:
 *   ORACLE_LUMO_ORDER  exactly lumo's tile-serial Xorshift stream (task.rs:27-76);
 *   ORACLE_WAVEFRONT   the per-path stream order the GPU implements.
 */
#ifndef LUMO_ORACLE_H
#define LUMO_ORACLE_H
#include "../include/lumo_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_WAVEFRONT = 0, ORACLE_LUMO_ORDER = 1 };

typedef struct {
    uint64_t aabb_tests;   /* BVH node + kd boundary slab tests */
    uint64_t kd_nodes;     /* kd interior node visits           */
    uint64_t tri_tests;    /* triangle tests (any kind)         */
    uint64_t closest_queries, shadow_queries;
} oracle_counters;

/* Render `n` tile tasks; `threads` worker threads (tasks are independent). */
int oracle_render_tiles(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                        const lumo_tile_task* tasks, size_t n, int mode, int threads,
                        lumo_tile_result* out, oracle_counters* counters);

/* Renderer::tone_map (tone_mapping.rs) for subsequent oracle_render_tiles calls:
 * kind LUMO_TONEMAP_NONE / CLAMP (arg = upper bound) / REINHARD. */
void oracle_set_tone_map(int kind, double arg);
/* Integrator for subsequent renders: LUMO_INTEGRATOR_PATH_TRACE or LUMO_INTEGRATOR_BDPT. */
void oracle_set_integrator(int integrator);
/* Acceleration structure of subsequent calls: 0 lumo's BVHs + kd-trees (default), 1 the wide BVH of
 * lumo_amd's LUMO_OPT_ACCEL = 1 (same structure as the upload builds, walk restated here). */
void oracle_set_accel(int accel);
/* Diagnostics: the wide BVH built for `scene`: info[8] = {ok, nodes, leaf triangle records, walk
 * stack need, node levels, objects root ref, lights root ref, 0}; non-null buffers (sized from a
 * first call with nulls) receive the nodes (128 B each), the records (10 doubles each) and the per
 * object / light BLAS roots. */
int oracle_wide_export(const lumo_scene_desc* scene, int64_t* info, void* nodes, double* tv, int32_t* obj_blas,
                       int32_t* light_blas);
/* SamplerType of subsequent renders (LUMO_SAMPLER_*, samplers.rs:6-17; default MultiJittered). */
void oracle_set_sampler(int sampler);
/* The points SamplerType::new(batch, samples, seed) yields (x, y interleaved, at most cap). */
int64_t oracle_sampler_points(uint64_t batch, uint64_t samples, uint64_t seed, double* out, int64_t cap);

/* Per-path record of the wavefront order for one task (for per-path parity tests):
 * out arrays sized (pixels * samples), pixel-major within each pass (pass s, pixel j). */
int oracle_trace_paths(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                       const lumo_tile_task* task, double* radiance4, double* lambda4,
                       double* raster2, uint64_t* depth, double* delta_per_pass);

/* Diagnostics: per-bounce record of path (pass, pixel) of one task (20 doubles each). */
int oracle_debug_trace(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                       const lumo_tile_task* task, int pass, int pixel, double* out, int* n_out);

/* Diagnostics: each ray's traversal counters (AABB, kd nodes, triangles) in cost3[3 i ..]. */
int oracle_trace_costs(const lumo_scene_desc* scene, const lumo_ray_soa* rays, size_t n, int any_hit,
                       uint32_t* cost3);
/* Scene::hit (any_hit = 0) or Scene::hit_light (any_hit != 0) for a batch of rays. */
int oracle_trace(const lumo_scene_desc* scene, const lumo_ray_soa* rays, size_t n,
                 lumo_hit_soa* hits, int any_hit, oracle_counters* counters);

/* BSDF probes at a surface point with ns = ng = +Z (front face), in world = shading space.
 * oracle_bsdf_sample: n samples of bsdf_sample(wo, lambda(u0), rand_u, rand_sq) with rng
 *   Xorshift::new(seed); ok[i] = 0 when the sample is None.
 * oracle_bsdf_eval: pdf and f (4 wavelengths of lambda4) for each wi.
 * oracle_furnace: white_furnace_tests.rs furnace_sample: mean f*cos/pdf over n samples. */
int oracle_bsdf_sample(const lumo_scene_desc* scene, int material, const double* wo, const double* lambda4,
                       size_t n, uint64_t seed, double* wi3, int* ok);
int oracle_bsdf_eval(const lumo_scene_desc* scene, int material, const double* wo, const double* lambda4,
                     const double* wi3, size_t n, double* pdf, double* f4);
int oracle_furnace(const lumo_scene_desc* scene, int material, const double* wo, size_t n, uint64_t seed,
                   double* out4);

/* Light sampling probes (object.rs:138-156, instance.rs:162-199): for light `light` seen from
 * point xo, oracle_light_sample draws n directions with sample_towards (rng Xorshift::new(seed));
 * oracle_light_pdf returns sample_towards_pdf for each direction whose ray hits the light
 * (Object::hit from xo), else 0. */
int oracle_light_sample(const lumo_scene_desc* scene, int light, const double* xo, size_t n, uint64_t seed,
                        double* wi3);
/* Math probes (spherical_utils / onb / complex / vec3 tests): see oracle.cpp oracle_math. */
int oracle_math(int op, const double* in, size_t n, double* out);

int oracle_light_pdf(const lumo_scene_desc* scene, int light, const double* xo, const double* wi3, size_t n,
                     double* pdf);

#ifdef __cplusplus
}
#endif
#endif
