/* lumo_amd: MI355X (gfx950) wavefront path tracer behind a C ABI.
 *
 * This header is the drop-in boundary for lumo's render hot path (ekarpp/lumo v0.6.1).
 * Every entry point names the reference interface it replaces (paths relative to the
 * lumo source tree).  Plain C: fixed-width integers, doubles, pointers and sizes only.
 * All calls return lumo_status (0 = OK); no exceptions cross the ABI.  A context is
 * bound to one GPU and owns all of its state (device buffers, streams, options, timers):
 * contexts share nothing mutable, so different contexts, on the same GPU or on different
 * ones, may be driven concurrently from different host threads; one context is used by one
 * thread at a time.
 */
#ifndef LUMO_AMD_H
#define LUMO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LUMO_ABI_VERSION 10

typedef int32_t lumo_status;
enum {
    LUMO_OK = 0,
    LUMO_ERR_INVALID = 1,     /* bad argument / malformed scene            */
    LUMO_ERR_NO_DEVICE = 2,   /* HIP device missing or not gfx950           */
    LUMO_ERR_HIP = 3,         /* HIP runtime error                          */
    LUMO_ERR_NO_SCENE = 4,    /* render/trace before lumo_scene_upload      */
    LUMO_ERR_NO_CAMERA = 5,   /* render before lumo_camera_set              */
    LUMO_ERR_UNSUPPORTED = 6, /* feature outside the implemented scope      */
    LUMO_ERR_OOM = 7
};

/* ---------------------------------------------------------------------------------
 * Flattened scene (the device image of lumo's Scene, src/tracer/scene.rs:17-29).
 * Produced on the host by lumo_amd's scene builder (or by lumo's own Rust Scene after
 * build(): the arrays below are exactly its BVH / kd-tree node arrays), copied to HBM
 * by lumo_scene_upload.  The caller owns all host arrays.
 * ------------------------------------------------------------------------------- */

/* Spectrum as sigmoid polynomial, f32 (spectrum.rs:14-19). */
typedef struct {
    float c0, c1, c2, scale;
} lumo_spectrum;

enum {
    LUMO_MAT_BLANK = 0,
    LUMO_MAT_LAMBERTIAN = 1,   /* BxDF::Lambertian (bxdf/scatter.rs:3-27)          */
    LUMO_MAT_LIGHT = 2,        /* Material::Light (material.rs:15, 223-234)         */
    LUMO_MAT_MF_DIFFUSE = 3,   /* BxDF::MfDiffuse    (bxdf/microfacet.rs:120-199)    */
    LUMO_MAT_MF_CONDUCTOR = 4, /* BxDF::MfConductor  (bxdf/microfacet.rs:62-118)     */
    LUMO_MAT_MF_DIELECTRIC = 5 /* BxDF::MfDielectric (bxdf/microfacet.rs:201-374)    */
};
enum { LUMO_MATF_CONSTANT_ETA = 1 /* DenseSpectrum::is_constant of eta (no dispersion) */ };

/* Textures (texture.rs:23-92, image.rs).  A material's albedo / ks / tf slot is its solid
 * spectrum when the slot's texture index is -1, else textures[index] evaluated at the hit's uv. */
enum {
    LUMO_TEX_SOLID = 0,        /* Texture::Solid                                        */
    LUMO_TEX_IMAGE = 1,        /* Texture::Image (image.rs:99-128, 170-184): texels[first..]  */
    LUMO_TEX_CHECKERBOARD = 2, /* Texture::Checkerboard(first, second, scale)           */
    LUMO_TEX_MARBLE = 3,       /* Texture::Marble(perlin[first], spec)                  */
    LUMO_TEX_MANDELBROT = 4    /* Texture::Mandelbrot                                   */
};
typedef struct {
    int32_t kind;          /* LUMO_TEX_*                                                 */
    int32_t width, height; /* IMAGE                                                      */
    int32_t first;         /* IMAGE: first texel; CHECKERBOARD: even cells; MARBLE: perlin */
    int32_t second;        /* CHECKERBOARD: odd cells                                    */
    int32_t pad0;
    double scale;          /* CHECKERBOARD                                               */
    lumo_spectrum spec;    /* SOLID / MARBLE colour; IMAGE: mean (Texture::power)        */
} lumo_texture;
/* Image<Normal> bump map (image.rs:131-166): normal_texels[3 * (first + x + y * width)..] */
typedef struct {
    int32_t width, height, first, pad0;
} lumo_normal_map;
/* Perlin noise lattice (perlin.rs): 256 unit normals and the x / y / z permutations */
typedef struct {
    double lattice[256][3];
    int32_t perm[3][256];
} lumo_perlin;

typedef struct {
    int32_t kind;       /* LUMO_MAT_*                                           */
    int32_t two_sided;  /* Light: emits from the back face too                   */
    int32_t illuminant; /* Light: index into dense_spectra                       */
    int32_t eta_idx;    /* microfacet: dense_spectra index of eta                */
    int32_t k_idx;      /* microfacet: dense_spectra index of k                  */
    int32_t flags;      /* LUMO_MATF_*                                           */
    double scale;       /* Light: emission scale                                 */
    double roughness;   /* microfacet: max(roughness, 1e-5)                      */
    lumo_spectrum albedo; /* Lambertian spectrum / Light texture / microfacet kd  */
    lumo_spectrum ks;
    lumo_spectrum tf;
    /* texture indices of albedo / ks / tf (-1: the solid spectrum above) and the bump map
     * (-1: none) of Material::Standard (material.rs:323-331) */
    int32_t albedo_tex, ks_tex, tf_tex, normal_map;
} lumo_material;

/* lumo BVH node (object/bvh.rs:18-26, bvh/node.rs:8-14), depth-first layout:
 * left child = index + 1, `right` = index of the right child or -1.
 * A leaf has count > 0: items[first .. first+count) are object indices. */
typedef struct {
    double bmin[3], bmax[3];
    int32_t right;
    int32_t first;
    int32_t count;
    int32_t pad0;
} lumo_bvh_node;

/* lumo kd-tree node (object/kdtree/node.rs:24-31), pre-order layout:
 * left child = index + 1; leaf: items[first .. first+count) are triangle indices
 * local to the owning object. */
typedef struct {
    double point;
    int32_t axis;
    int32_t right;
    int32_t leaf;
    int32_t first;
    int32_t count;
    int32_t pad0;
} lumo_kd_node;

enum {
    LUMO_OBJ_KDMESH = 0,    /* KdTree<Triangle> (TriangleMesh::new, triangle_mesh.rs:46-60) */
    LUMO_OBJ_RECTANGLE = 1, /* Rectangle (object/rectangle.rs): 2-triangle kd mesh + uv/sampling */
    LUMO_OBJ_TRIANGLE = 2,  /* a single Triangle (object/triangle.rs), e.g. an emissive OBJ face
                               added as a light (parser/obj.rs:93-103)                       */
    LUMO_OBJ_SPHERE = 3     /* Sphere at the local origin (object/sphere.rs), e.g. the
                               environment light of Scene::build (scene.rs:33-52)            */
};

/* Instance transform (object/instance.rs, math/transform.rs): row-major 4x4 local->world `m`,
 * its inverse `inv`, and the normal transform (transpose of inv's 3x3, Transform::to_normal). */
typedef struct {
    double m[16];
    double inv[16];
    double nrm[9];
    double pad0;
} lumo_transform;

typedef struct {
    int32_t type;      /* LUMO_OBJ_* of the shape                        */
    int32_t material;  /* material of the mesh (KdTree::material)        */
    int32_t kd_root;   /* index of the root in kd_nodes (-1: TRIANGLE)   */
    int32_t tri_base;  /* first triangle of this object in triangles[]   */
    int32_t item_base; /* kd leaf item lists live in kd_items[item_base..] */
    int32_t num_tris;
    int32_t xform;     /* Instance: index into transforms[], else -1     */
    int32_t material_override; /* Instance material (instance.rs:96-98) or -1 */
    double bmin[3], bmax[3]; /* kd boundary in the shape's own space (KdTree::boundary) */
    double origin[3], b0[3], b1[3]; /* Rectangle parameters (rectangle.rs:6-13) */
    double area;       /* Sampleable::area of the shape (own space)      */
    double radius;     /* Sphere radius                                  */
} lumo_object;

typedef struct {
    int32_t v[3];   /* vertex indices into vertices[]                 */
    int32_t n[3];   /* shading-normal indices or -1                   */
    int32_t t[3];   /* uv indices or -1                               */
    int32_t material;
} lumo_triangle;

typedef struct {
    /* geometry */
    int32_t num_vertices, num_normals, num_uvs, num_triangles;
    const double* vertices; /* xyz f64 */
    const double* normals;  /* xyz f64 */
    const double* uvs;      /* uv f64  */
    const lumo_triangle* triangles;
    /* per-object kd-trees */
    int32_t num_kd_nodes, num_kd_items;
    const lumo_kd_node* kd_nodes;
    const int32_t* kd_items;
    /* objects BVH (Scene::objects) */
    int32_t num_objects, num_object_nodes, num_object_items;
    const lumo_object* objects;
    const lumo_bvh_node* object_nodes;
    const int32_t* object_items;
    /* lights BVH (Scene::lights) + power alias table (bvh.rs:105-191) */
    int32_t num_lights, num_light_nodes, num_light_items;
    const lumo_object* lights;
    const lumo_bvh_node* light_nodes;
    const int32_t* light_items;
    const double* alias_prob;  /* alias_table[i].0 */
    const int32_t* alias_idx;  /* alias_table[i].1 */
    const double* alias_pdf;   /* alias_pdf[i]     */
    /* materials and 95-bin dense spectra (dense_spectrum.rs) */
    int32_t num_materials, num_dense_spectra;
    const lumo_material* materials;
    const double* dense_spectra; /* num_dense_spectra x 95 */
    /* instance transforms referenced by lumo_object.xform */
    int32_t num_transforms, pad1;
    const lumo_transform* transforms;
    /* textures (texture.rs), their texels (Spectrum per pixel), bump maps, Perlin lattices */
    int32_t num_textures, num_texels;
    const lumo_texture* textures;
    const lumo_spectrum* texels;
    int32_t num_normal_maps, num_normal_texels;
    const lumo_normal_map* normal_maps;
    const double* normal_texels; /* xyz f64 */
    int32_t num_perlin, pad2;
    const lumo_perlin* perlin;
} lumo_scene_desc;

/* Camera (camera.rs:17-38, CameraConfig): world_to_camera, screen_to_raster and
 * camera_to_screen transforms as (m, inv) row-major 4x4 pairs.  Camera::Perspective or
 * Camera::Orthographic (camera.rs:127-132; generate_ray :257-268).  lumo's orthographic camera
 * has no importance functions (camera.rs:348-351 `unimplemented!()`), so BDPT with it is
 * LUMO_ERR_UNSUPPORTED, as it panics in lumo. */
typedef struct {
    double world_to_camera[2][16];
    double screen_to_raster[2][16];
    double camera_to_screen[2][16];
    double lens_radius, focal_length;
    int64_t width, height;
    int32_t orthographic; /* 0 = Perspective, 1 = Orthographic */
    int32_t illuminant;   /* dense_spectra index used for white balance */
    double white_balance[9];   /* ColorSpace::wb_matrix (space.rs:144-151), row-major */
    double xyz_to_rgb[9];      /* colour space XYZ->RGB (default DCI-P3, space.rs:51-54) */
    double filter_radius, filter_sigma; /* PixelFilter::Gaussian (filter.rs:20-24) */
} lumo_camera_desc;

/* RenderTask (renderer/task.rs:86-104): one tile x one sample batch. */
typedef struct {
    uint64_t px_min[2], px_max[2]; /* tile [px_min, px_max) in raster space */
    uint64_t batch;                /* sample batch index (256 spp per batch) */
    uint64_t samples;              /* samples in this batch                  */
    uint64_t total_samples;        /* Renderer::num_samples                  */
    uint64_t seed;                 /* task seed from the renderer stream     */
} lumo_tile_task;

/* RenderTaskResult (renderer/task.rs:106-116) + its FilmTile pixels (film/tile.rs).
 * `rgb_w` is caller-allocated: 4 doubles (sum w*r, w*g, w*b, sum w) per pixel of the
 * tile, row-major over [px_min, px_max). */
/* A light-tracing splat of BDPT (FilmSample with splat = true): filtered RGB added to the
 * full-frame splat buffer at pixel (x, y) (film/tile.rs:96-101, film.rs:167-170). */
typedef struct {
    uint32_t x, y;
    double rgb[3];
} lumo_splat;

typedef struct {
    double* rgb_w;
    uint64_t num_camera_rays;
    uint64_t num_rays;       /* sum of FilmSample.cost (path depth), task.rs:65 */
    uint64_t num_queries;    /* closest-hit + shadow visibility queries issued  */
    /* BDPT splats of this task in lumo's order; caller-allocated `splat_cap` entries.  On
     * return num_splats is the count produced; a count above splat_cap fails the call with
     * LUMO_ERR_OOM (retry with a larger buffer). */
    lumo_splat* splats;
    uint64_t splat_cap;
    uint64_t num_splats;
} lumo_tile_result;

enum { LUMO_RNG_WAVEFRONT = 0, LUMO_RNG_LUMO_ORDER = 1 };
/* SamplerType (samplers.rs:6-17), the pixel sampler of Renderer::sampler (renderer.rs:89-93).
 * Sobol draws from a 10-bit sequence (samplers/sobol_seq.rs: SOBOL_MAX_LEN 1023): more than 1023
 * samples per pixel panic in lumo and are LUMO_ERR_INVALID here. */
enum { LUMO_SAMPLER_MULTI_JITTERED = 0, LUMO_SAMPLER_UNIFORM = 1, LUMO_SAMPLER_JITTERED = 2, LUMO_SAMPLER_SOBOL = 3 };
enum { LUMO_INTEGRATOR_PATH_TRACE = 0, LUMO_INTEGRATOR_BDPT = 1 };

typedef struct {
    int32_t integrator; /* LUMO_INTEGRATOR_*                              */
    int32_t rng_mode;   /* LUMO_RNG_WAVEFRONT (GPU); lumo-order: oracle only */
    int32_t max_paths;  /* cap on paths in flight (0 = all pixels of the call) */
    int32_t tone_map;   /* LUMO_TONEMAP_* applied per sample before the film (task.rs:73-76)  */
    double tone_arg;    /* ToneMap::Clamp upper bound                                          */
    /* BDPT only.  max_vertices: storage per subpath (0 = 128).  A sample whose subpath is longer
     * is re-run with storage for lumo's maximum depth (1025); more than 4096 such samples in one
     * pass fail the call with LUMO_ERR_UNSUPPORTED (never truncated).  splat_film: optional
     * row-major width x height x 3 array; when a task's result has no `splats` list, its
     * light-tracing taps are summed into it (film.rs:167-170; summation order unspecified, as
     * lumo's tile completion order). */
    int32_t max_vertices;
    int32_t sampler;    /* LUMO_SAMPLER_* (0 = MultiJittered, lumo's default)                  */
    double* splat_film;
} lumo_render_cfg;
enum { LUMO_TONEMAP_NONE = 0, LUMO_TONEMAP_CLAMP = 1, LUMO_TONEMAP_REINHARD = 2 }; /* tone_mapping.rs */

/* Ray batch for traversal-only queries (parity + micro-benchmarks). */
typedef struct {
    const double* origin; /* n x 3 */
    const double* dir;    /* n x 3 */
    const double* t_max;  /* n (closest: ignored, INF) */
    const int32_t* light; /* n: light index for visibility queries (any_hit mode) */
} lumo_ray_soa;

typedef struct {
    double* t;       /* closest: hit t (INF on miss); visibility: light t or INF if occluded */
    int32_t* kind;   /* 0 miss, 1 object, 2 light                                      */
    int32_t* object; /* object / light index                                           */
    int32_t* prim;   /* triangle index (global)                                        */
} lumo_hit_soa;

/* Per-stage device time (HIP events; only with LUMO_OPT_TIMING on), launch
 * counts, query counts and traversal counters (AABB slab tests, kd split-node visits,
 * triangle tests) of the closest-hit [0] and shadow / connection [1] kernels, summed over
 * renders.  BDPT: CLOSEST + SHADE are the subpath walks, RESOLVE the re-runs + fold, BD_* the
 * connection items.  samples_{nan,neg,large} count the camera samples whose radiance has a NaN,
 * a negative or a > 1000 component (the debug_assertions checks of tone_mapping.rs:42-56,
 * counted instead of recoloured; the image is unchanged). */
enum { LUMO_STAGE_CAMERA = 0, LUMO_STAGE_CLOSEST, LUMO_STAGE_SHADE, LUMO_STAGE_SHADOW, LUMO_STAGE_RESOLVE,
       LUMO_STAGE_FINISH, LUMO_STAGE_FILM, LUMO_STAGE_RING, LUMO_STAGE_BD_TRACE_A, LUMO_STAGE_BD_EVAL_A,
       LUMO_STAGE_BD_VIS, LUMO_STAGE_BD_PATHS, LUMO_STAGE_COUNT };
typedef struct {
    double kernel_ms[LUMO_STAGE_COUNT];
    uint64_t launches[LUMO_STAGE_COUNT];
    uint64_t closest_queries, shadow_queries, bounces;
    uint64_t aabb_tests[2], kd_nodes[2], tri_tests[2];
    uint64_t samples_nan, samples_neg, samples_large;
    /* shadow queries (included in shadow_queries) whose contribution is zero whatever the
     * visibility: the record's BSDF pdf is 0, so mis_sample returns 0 before using the hit
     * (integrator.rs:146); the device answers them without traversing the scene. */
    uint64_t shadow_resolved;
    /* closest queries (included in closest_queries) run by the path tracer's tail kernel past
     * the first bounce it takes: > 0 when the device switched a pass to the tail kernel (ABI 9) */
    uint64_t tail_queries;
    /* bounces whose closest-hit rays were sorted before their walks (LUMO_OPT_RAY_SORT; ABI 10) */
    uint64_t sorted_bounces;
} lumo_stats;

/* Per-path dump of one task (test hook for per-path parity): arrays sized samples x pixels
 * (pass-major, pixel raster order within the tile); delta has one entry per pass. */
typedef struct {
    double* radiance;  /* 4 per path */
    double* lambda_;   /* 4 per path */
    double* raster;    /* 2 per path */
    uint64_t* depth;
    double* delta;
} lumo_path_dump;

/* --- context ---------------------------------------------------------------------- */
/* Replaces: ThreadPool::new + RenderTaskExecutor::new (pool.rs:17-38, task.rs:12-21). */
lumo_status lumo_create(int device, void** ctx_out);
void lumo_destroy(void* ctx);
const char* lumo_status_str(lumo_status st);
int lumo_abi_version(void);
/* Number of visible GPUs (0 when the HIP runtime has none). */
int lumo_device_count(void);

/* Replaces: Renderer::new(scene, ...) -> scene.build() + Arc<Scene> (renderer.rs:40-63). */
lumo_status lumo_scene_upload(void* ctx, const lumo_scene_desc* scene);
/* Replaces: Arc<Camera> shared with the executor (task.rs:4-10). */
lumo_status lumo_camera_set(void* ctx, const lumo_camera_desc* camera);

/* Replaces: Executor<RenderTask, RenderTaskResult>::exec (pool.rs:6-8, task.rs:24-82),
 * batched: all n tasks are rendered as one wavefront. */
lumo_status lumo_render_tiles(void* ctx, const lumo_tile_task* tasks, size_t n,
                              const lumo_render_cfg* cfg, lumo_tile_result* out);

/* Replaces: Scene::hit (scene.rs:119-147) when any_hit == 0, and
 * Scene::hit_light (scene.rs:165-189) when any_hit != 0.  Host buffers in and out. */
lumo_status lumo_trace(void* ctx, const lumo_ray_soa* rays, size_t n, lumo_hit_soa* hits,
                       int any_hit);

lumo_status lumo_stats_get(void* ctx, lumo_stats* stats);
lumo_status lumo_stats_reset(void* ctx);
/* Busy time of a set of stages (bit k = LUMO_STAGE k) since the last reset, with timing on: the
 * length of the union of their launches' intervals.  kernel_ms sums launch durations, which counts
 * twice the time that launches on concurrent streams overlap (pipelined passes); this does not. */
lumo_status lumo_stats_busy_ms(void* ctx, uint32_t stage_mask, double* ms);
/* ---------------------------------------------------------------------------------
 * Per-context execution options.  Every option changes only how the work is scheduled on the
 * device, never a result: all values give bit-identical films, counters and traces.  Options are
 * state of the context, so contexts (on one GPU or on several) driven from different host
 * threads do not interfere (lumo's executors share nothing but the task receiver, pool.rs:17-38).
 * A context starts from the defaults below, overridden by the environment variable named beside
 * each (read once, in lumo_create).  Options marked "upload" take effect at the next
 * lumo_scene_upload.  lumo_set_option returns LUMO_ERR_INVALID for an unknown option or a value
 * out of range.
 * ------------------------------------------------------------------------------- */
enum {
    LUMO_OPT_TIMING = 0,       /* per-launch HIP-event timing of every stage: 0 / 1 (LUMO_TIMING, 0)   */
    LUMO_OPT_LDS_STAGING,      /* stage a scene of <= 48 KiB whole in LDS: 0 / 1 (LUMO_LDS, 1)          */
    LUMO_OPT_TOP_STAGING,      /* TOP staging of larger scenes: 0 / 1 (LUMO_TOP, 1)                    */
    LUMO_OPT_FUSED,            /* n_shadow = 1: -1 fused bounce when LDS-staged, 0 three kernels,
                                  1 fused (LUMO_FUSED, -1)                                          */
    LUMO_OPT_TAIL_BELOW,       /* n_shadow = 1: tail kernel below this many live paths, 0 never
                                  (LUMO_TAIL, 65536)                                               */
    LUMO_OPT_PIPELINE,         /* passes overlapped: 0 off, fused bounces 1-3 head streams, split
                                  schedule on when > 0 (LUMO_PIPELINE, 3)                            */
    LUMO_OPT_HEADS,            /* fused pipeline: bounces per pass on its head stream, 0 auto
                                  (LUMO_HEADS, 0)                                                   */
    LUMO_OPT_MERGE_PASSES,     /* fused and split pipelines: consecutive passes whose cameras and
                                  head bounces (those before Russian roulette) run as one queue,
                                  0 auto, 1-8 (LUMO_MERGE, 0)                                        */
    LUMO_OPT_DYN_FETCH,        /* fused bounce: blocks fetch paths from a counter: 0 / 1 (LUMO_DYN, 0)*/
    LUMO_OPT_BOUNCE_THREADS,   /* fused bounce: threads per block 64 / 128 / 256
                                  (LUMO_BOUNCE_THREADS, 256)                                        */
    LUMO_OPT_SPLIT_PIPE,       /* split schedule: units in flight 1-4 (LUMO_SPLIT_PIPE, 4)           */
    LUMO_OPT_SPLIT_GROUPS,     /* split schedule: independent task groups 1-4 (LUMO_SPLIT_GROUPS, 2) */
    LUMO_OPT_BDPT_TAIL,        /* BDPT: walk-tail kernel below this many live subpaths, 0 never
                                  (LUMO_BDPT_TAIL, 65536)                                           */
    LUMO_OPT_BOUNCE_AHEAD,     /* bounces enqueued ahead of the host's count snapshots 1-63
                                  (LUMO_BOUNCE_AHEAD, 3)                                            */
    LUMO_OPT_LDS_GRID,         /* grid cap of LDS-staged kernels (LUMO_LDS_GRID, 1.5 x CUs = 384)    */
    LUMO_OPT_TOP_GRID,         /* grid cap of TOP kernels (LUMO_TOP_GRID, half the CU count = 128)   */
    LUMO_OPT_TOP_KB,           /* upload: TOP set budget in KiB, <= the CU's LDS (LUMO_TOP_KB)       */
    LUMO_OPT_KD_LDS,           /* upload: kd stack entries per thread in LDS in TOP kernels
                                  (LUMO_KD_LDS, 8)                                                  */
    LUMO_OPT_STACK_CLASS,      /* upload: kd stack class override, 0 auto; never below the scene's
                                  need (LUMO_STACK_CLASS, 0)                                        */
    LUMO_OPT_FULL_KERNELS,     /* upload: general feature kernels even for lean scenes: 0 / 1
                                  (LUMO_FULL_KERNELS, 0)                                            */
    LUMO_OPT_POISON,           /* debug: fill every newly allocated device buffer with 0xFF bytes,
                                  so a read of a buffer before its first write shows (LUMO_POISON, 0)*/
    LUMO_OPT_TAIL_PRIORITY,    /* fused pipeline: the stream of the passes' tails, films and rings (the
                                  chain each pass's Russian roulette waits on) at high priority: 0 / 1
                                  (LUMO_TAIL_PRIORITY, 0)                                           */
    LUMO_OPT_TOP_KD,           /* upload: the TOP set's spare LDS holds the top treelets of the
                                  largest kd tree: 0 / 1 (LUMO_TOP_KD, 1)                           */
    LUMO_OPT_TAIL_BOUNCES,     /* fused pipeline: fused bounces per pass the tail stream runs before the
                                  tail kernel, -1 auto (2 for one-pass units, 0 for merged ones), 0-16
                                  (LUMO_TAIL_BOUNCES, -1)                                           */
    LUMO_OPT_FILM_FIRST,       /* fused pipeline, film on the tail stream: the unit's film before its
                                  last ring: 0 / 1 (LUMO_FILM_FIRST, 0)                             */
    LUMO_OPT_BDPT_TOP,         /* BDPT connection visibility (k_bdpt_vis) of scenes too large to stage
                                  whole reads the TOP set and kd stack columns from LDS: 0 / 1
                                  (LUMO_BDPT_TOP, 1)                                                */
    LUMO_OPT_BDPT_GROUPS,      /* BDPT: task groups rendered as concurrent chains of passes on their own
                                  streams, 1-4 (LUMO_BDPT_GROUPS, 2; ABI 9)                          */
    LUMO_OPT_RAY_SORT,         /* three-kernel bounces: the closest-hit rays of a bounce radix-sorted
                                  before their walks: 0 off, 1 direction octant major, 2 origin cell
                                  major, -1 auto (1 for kd stack class >= 32) (LUMO_RAY_SORT, -1; ABI 9)*/
    LUMO_OPT_ACCEL,            /* upload: acceleration structure the walks use.  0 lumo's own (the
                                  objects / lights BVHs, bvh.rs, and per-mesh kd-trees, kdtree.rs;
                                  bit-exact with the reference), 1 wide (a 4-wide SAH BVH over all
                                  primitives, nearest child first; same hit semantics except ties and
                                  BDPT's visible()) (LUMO_ACCEL, 0; ABI 10)            */
    LUMO_OPT_COUNT
};
lumo_status lumo_set_option(void* ctx, int32_t option, int64_t value);
lumo_status lumo_get_option(void* ctx, int32_t option, int64_t* value);

/* The schedule the last lumo_render_tiles call used (after its last max_paths chunk): which
 * pass loop ran and with how many streams, units, groups and merged passes.  Lets callers and
 * tests check that a requested schedule was not cut back (free HBM bounds the split schedule's
 * units in flight). */
enum { LUMO_SCHED_SEQUENTIAL = 0, LUMO_SCHED_FUSED_PIPELINE = 1, LUMO_SCHED_SPLIT_PIPELINE = 2,
       LUMO_SCHED_BDPT_GROUPS = 3 /* ABI 9 */ };
typedef struct {
    int32_t schedule;        /* LUMO_SCHED_*                                               */
    int32_t head_streams;    /* fused pipeline: head streams                               */
    int32_t head_bounces;    /* fused pipeline: bounces per pass on the head stream        */
    int32_t merged_passes;   /* fused / split pipeline: passes per head unit               */
    int32_t units_in_flight; /* split pipeline: (group, pass) units in flight; BDPT groups  */
    int32_t task_groups;     /* split pipeline / BDPT groups: independent task groups      */
    int32_t fused;           /* 1: fused bounce kernel, 0: three kernels per bounce         */
    int32_t tail_bounces;    /* fused pipeline: fused bounces per pass on the tail stream   */
} lumo_schedule_info;
lumo_status lumo_last_schedule(void* ctx, lumo_schedule_info* info);

/* Test hook: render one task in the wavefront order and dump every path. */
lumo_status lumo_debug_paths(void* ctx, const lumo_tile_task* task, lumo_path_dump* dump);
/* Integrator of lumo_debug_paths (LUMO_INTEGRATOR_*; BDPT splats are not collected there). */
lumo_status lumo_debug_set_integrator(void* ctx, int integrator);
/* Pixel sampler of lumo_debug_paths (LUMO_SAMPLER_*). */
lumo_status lumo_debug_set_sampler(void* ctx, int sampler);
/* Diagnostics: per-bounce record (20 doubles per bounce, at most 64 bounces) of the path of
 * `pixel` in sample pass `pass` of `task`; *n_out = number of bounces recorded. */
lumo_status lumo_debug_trace(void* ctx, const lumo_tile_task* task, int pass, int pixel, double* out,
                             int* n_out);
/* Kernel variant selected for the uploaded scene: kd stack class, bytes of scene staged in LDS
 * (0: no staging), feature class (1: instances / spheres / triangle lights / microfacet
 * materials), shadow rays per bounce (scene.rs:90-92).  Scenes too large to stage whole stage
 * their TOP set in the closest-hit and visibility kernels: top_bytes of LDS per block (0: none),
 * holding the first top_object_nodes / top_light_nodes nodes (breadth-first: the top levels) of
 * the objects / lights BVH, the object items and the objects' traversal records. */
typedef struct {
    int32_t stack_class, lds_bytes, full_kernels, n_shadow;
    int32_t top_bytes, top_object_nodes, top_light_nodes;
    int32_t top_kd_nodes; /* kd nodes of the largest kd tree (its top treelets) in the TOP set */
    int32_t top_shm;      /* LDS per TOP block: the TOP set + the kd stack columns, within
                             LUMO_OPT_TOP_KB (ABI 9)                                          */
    /* ABI 10: the acceleration structure the uploaded scene is walked with (LUMO_OPT_ACCEL: 0 lumo,
     * 1 wide; 0 also when wide was asked for and the build refused the scene, e.g. a tree needing
     * more than 64 walk stack entries) and, for wide, its nodes, leaf triangle records, deepest
     * walk stack, node levels and the nodes of its TOP set (a breadth-first prefix) */
    int32_t accel, wide_nodes, wide_tris, wide_stack, wide_depth, top_wide_nodes;
} lumo_scene_info_t;
lumo_status lumo_scene_info(void* ctx, lumo_scene_info_t* info);
/* Diagnostics: one coalesced 8-B-per-lane read stream and one write stream over n doubles
 * (kernels k_calib_read8 / k_calib_write8), to calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for
 * the access width of the path kernels. */
lumo_status lumo_debug_stream(void* ctx, size_t n);
/* Diagnostics (ABI 10): the device's exclusive prefix sum (device/scan.h, the BDPT item lists' scan)
 * of n host uint32 counts into out. */
lumo_status lumo_debug_scan(void* ctx, const uint32_t* in, uint32_t* out, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* LUMO_AMD_H */
