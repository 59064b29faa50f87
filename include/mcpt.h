/* mcpt.h — C ABI of the MI355X path tracer (libmcpt.so).
 *
 * Drop-in boundary for the reference's hot path.  Two halves:
 *
 *  1. Device renderer — replaces the GL program `prg_ray` (raytracer.vert +
 *     raytracer_func.frag + tp/<variant>.frag + main.frag), its texture/uniform ABI
 *     and the additive RGB32F FBO of MontecarloGPU/montecarlo.cpp:384-386, 408-477.
 *  2. Host scene producer — replaces ScenePrimitives / BVH_KDtree / BVH_GPU_Scene
 *     (bvh_gpu/scene.h:75-185, bvh.h:10-60, gpu_bvh_scene.h:35-121) and the canonical
 *     camera (easycppogl/camera.cpp:53-95 + montecarlo.cpp:388-389, 404-405, 439-440).
 *
 * Conventions: plain pointers and sizes, no torch types.  Matrices are 16 floats,
 * column-major (GL / Eigen storage).  Images are H rows × W pixels × RGB f32, row 0 =
 * bottom (GL window coordinates).  Every function returns an int status: 0 = ok,
 * negative = error (see mcpt_status); mcpt_error_string() describes it.  The caller
 * owns host arrays; the library owns device copies.  One context per GPU; calls on
 * one context are not thread-safe; contexts on different GPUs may run concurrently.
 * There is NO CPU fallback: every render call runs the HIP kernel or fails.
 */
#ifndef MCPT_H_
#define MCPT_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mcpt_status {
  MCPT_OK = 0,
  MCPT_ERR_INVALID_ARG = -1,
  MCPT_ERR_NO_SCENE = -2,
  MCPT_ERR_NO_TARGET = -3,
  MCPT_ERR_HIP = -4,         /* a HIP runtime call failed (no GPU, launch failure ...) */
  MCPT_ERR_NOT_FINALIZED = -5,
  MCPT_ERR_BAD_SCENE = -6,
};

/* integrator variants: the SrcLoader list of MontecarloGPU/montecarlo.cpp:27 */
enum mcpt_variant {
  MCPT_MONTECARLO = 0,       /* tp/montecarlo.frag        */
  MCPT_MAT = 1,              /* tp/montecarlo_mat.frag    */
  MCPT_MAT_TR = 2,           /* tp/montecarlo_mat_tr.frag */
};

/* BVH traversal strategy of the kernel (same results, different speed) */
enum mcpt_traversal {
  MCPT_TRAVERSAL_AUTO = 0,   /* measured: after a scene upload, launches of >= 2^24 samples time
                                the schedule candidates twice each (per-lane walks with 1/2/4 pass
                                segments per work item, the wave-coherent walk for BVH depth < 8,
                                the deep-BVH knobs at 4/8 segments for depth >= 8; never the stream
                                schedule); later launches of that shape use the fastest */
  MCPT_TRAVERSAL_LANE = 1,   /* each lane walks its own DFS (divergent, vector loads) */
  MCPT_TRAVERSAL_WAVE = 2,   /* the wave walks the union of its lanes' DFS orders (scalar loads) */
  MCPT_TRAVERSAL_STREAM = 3, /* wavefront schedule: a pool of path slots in HBM, iterations of one
                                trace kernel (persistent waves, a lane takes the next queued ray as
                                soon as its walk ends) and one shade kernel.
                                Variant montecarlo.frag, scenes without meshes, bounces > 0; other
                                renders run the per-lane walk.  mcpt_render returns once the
                                iterations have been issued (it waits on the device while it issues
                                them, to know when the slots are done).  Only when selected: AUTO
                                never times it (5 % behind the megakernel on the deepest BVH) */
};

/* algorithmic-byte event counters, index order */
enum mcpt_event {
  MCPT_EV_NODE = 0, MCPT_EV_LEAF, MCPT_EV_PRIM, MCPT_EV_CAND, MCPT_EV_GEOM, MCPT_EV_COLMAT,
  MCPT_EV_SAMPLE, MCPT_EV_TRAV, MCPT_EV_MESH, MCPT_EV_TRI, MCPT_EV_MGEOM, MCPT_EV_COUNT
};

typedef struct mcpt_ctx mcpt_ctx;
typedef struct mcpt_scene mcpt_scene;

const char* mcpt_error_string(int status);
int mcpt_version(void);
/* Which diagnostic build this library is (never a timed build): bit MCPT_BUILD_CHECKED the
 * bounds-checked build (make checked: out-of-range work-item / split / segment indices are counted
 * and skipped, every sub-launch is waited for and a fault or count fails the render call with the
 * sub-launch named), MCPT_BUILD_STAMPS / _LANESTATS / _BLOCKTIMES the instrumented builds,
 * MCPT_BUILD_DRIVER_MATH a GL-driver-arithmetic build.  0: the shipped library. */
enum { MCPT_BUILD_CHECKED = 1, MCPT_BUILD_STAMPS = 2, MCPT_BUILD_LANESTATS = 4, MCPT_BUILD_BLOCKTIMES = 8,
       MCPT_BUILD_DRIVER_MATH = 16 };
int mcpt_build_flags(void);

/* ---------------------------------------------------------------------------------
 * 1. device renderer
 * --------------------------------------------------------------------------------- */

/* create a context on HIP device `device_ordinal` (replaces GLViewer ctx + prg_ray) */
int mcpt_create(int device_ordinal, mcpt_ctx** out);
int mcpt_destroy(mcpt_ctx* ctx);

/* Upload a finalized scene in the reference's texture layouts:
 *   prims  : n_prims × 64 f32 (16 RGBA texels per PrimData, scene.h:64-73)
 *   nodes  : (2^(depth+1)-1) × 6 f32 (bbmin.xyz, bbmax.xyz)  — tex_bb, gpu_bvh_scene.cpp:39-41
 *   leaves : 2^depth i32 (prim index or -1)                   — tex_ind, gpu_bvh_scene.cpp:143-144
 * Replaces BVH_GPU_Scene::finalize's Texture2D uploads (gpu_bvh_scene.cpp:143-160) and
 * the uniforms nb_prims(1), bvh_depth(2), nb_emissives(20).  Transforms must be affine
 * (row 3 = 0,0,0,1: the shader only uses .xyz).  Limit: n_prims < 2^24 (MCPT_ERR_INVALID_ARG
 * otherwise) — the kernel packs a hit's primitive index, shape and face into one 32-bit word
 * (shape << 28 | face << 24 | index), which keeps the walk's hit record in 7 registers.
 * Synchronous. */
int mcpt_upload_scene(mcpt_ctx* ctx, const float* prims, int n_prims, const float* nodes,
                      const int* leaves, int depth, int nb_emissives);

/* Upload the scene's meshes (replaces the tex_tri_/tex_p_/tex_n_ textures and the per-mesh
 * BVH rows of tex_bb_/tex_ind_, gpu_bvh_scene.cpp:87-118, 160-186).  Layouts: see
 * mcpt_scene_get_mesh_buffers.  n_meshes = 0 removes them.  Call after mcpt_upload_scene;
 * a CODE_MESH primitive's record holds its mesh id (texel 12 .y, "mesh_line").  Limits (else
 * MCPT_ERR_BAD_SCENE): BVH depth <= 24 per mesh, and the device's mesh BVH records (64 B per
 * internal node + 64 B per leaf, all meshes) within 4 GiB — the walk addresses them by 32-bit
 * offsets — i.e. about 33 M triangles in all. */
int mcpt_upload_meshes(mcpt_ctx* ctx, int n_meshes, const int* info, int n_nodes, const float* nodes, int n_leaves,
                       const int* leaves, int n_tris, const int* tris, int n_verts, const float* verts,
                       const float* normals);

/* uniform flat_face (raytracer_func.frag:26, location 3): flat triangle normals instead of
 * the area-weighted vertex normals.  The reference never sets it (false); default 0. */
int mcpt_set_flat_face(mcpt_ctx* ctx, int flat_face);

/* Set the framebuffer (replaces FBO RGB32F + resize_ogl, montecarlo.cpp:384-386, 616-626).
 * Row-band sharding for multi-GPU: this context renders global rows y whose band
 * (y / band_rows) satisfies band % world == rank; its accumulator holds only those
 * "local" rows, in increasing y.  Single GPU: band_rows = any > 0, world = 1, rank = 0.
 * Allocates and zeroes the accumulator; pass count reset to 0.  MCPT_ERR_INVALID_ARG when this
 * context's local rows × W reach 2^31 pixels (the kernels index a shard with 32-bit ints). */
int mcpt_set_target(mcpt_ctx* ctx, int W, int H, int band_rows, int world, int rank);
int mcpt_local_rows(mcpt_ctx* ctx, int* n_local_rows);
/* Explicit shard: this context renders the n_rows global rows rows[0..n_rows) (distinct, in
 * [0, H)), local row i = global row rows[i]; the accumulator holds n_rows × W pixels.
 * Results per pixel do not depend on the partition. */
int mcpt_set_target_rows(mcpt_ctx* ctx, int W, int H, const int* rows, int n_rows);
/* The balanced multi-GPU partition: bands of band_rows rows dealt to ranks
 * period by period with a rotation (period j: rank r takes band j·world + (r+j) mod world),
 * the rows after the last whole period dealt singly; every rank gets floor(H/world) or
 * ceil(H/world) rows.  Writes rank's rows (increasing; rows_out may be NULL to query the
 * count) and their number.  Host-only (no device). */
int mcpt_balanced_rows(int H, int world, int rank, int band_rows, int* rows_out, int* n_out);
/* The context's global row ids of its local rows (n_local_rows ints). */
int mcpt_local_row_ids(mcpt_ctx* ctx, int* rows_out);

/* Accumulate passes first_pass .. first_pass+n_passes-1 into the accumulator (the
 * glDrawArrays loop of montecarlo.cpp:454-466 with blend ONE/ONE).  Summation order
 * (DESIGN.md §3.3): per pixel, passes are summed from 0 within each chunk of 32
 * consecutive absolute pass numbers ((pass-1)/32), and chunk sums are added to the
 * accumulator in chunk order — results are identical for any GPU count and for any
 * split of a pass range into calls at multiples of 32.  Uniform ABI:
 * invPV(10), invV(6), numero_pass(4) = pass index, date(5), NB_BOUNCES(21),
 * refract_ind(24); variant = tp/ shader.  Asynchronous on the context's stream.
 * Scheduling (never the bits): a launch of >= 4,096 work items times its items
 * and the next launch of the same shape runs them costliest first (a device sort on the
 * context's stream: no host wait; env MCPT_ITEM_ORDER=0 turns it off); launches whose work items
 * hold several pass segments run the last workgroup-generation of that order one segment per
 * workgroup (env MCPT_TAIL_PIECES=0 turns that off); in mesh scenes, launches of whole 32-pass
 * chunks also run their costliest items in 4 pass ranges side by side (env MCPT_SPLIT_ITEMS=0
 * turns that off).  Device memory for it: 20 B per work item, and 100 MB of per-pass values
 * once a mesh launch splits items. */
int mcpt_render(mcpt_ctx* ctx, const float* invPV, const float* invV, int first_pass,
                int n_passes, float date, int bounces, float refract_ind, int variant);

/* Same, with the counting build of the kernel: adds MCPT_EV_COUNT event totals into
 * events[] (algorithmic bytes = Σ events × mcpt_event_bytes).  Synchronous. */
int mcpt_render_counted(mcpt_ctx* ctx, const float* invPV, const float* invV, int first_pass,
                        int n_passes, float date, int bounces, float refract_ind, int variant,
                        unsigned long long* events);
int mcpt_event_bytes(int event);

#define MCPT_DEBUG_SLOTS 64
/* Diagnostics: read the first min(n_slots, MCPT_DEBUG_SLOTS) of the context's device counter
 * slots into `out` (which holds n_slots values; the first MCPT_EV_COUNT are the event counters)
 * and optionally zero them all.  The counting launches and diagnostic builds (-DMCPT_STAMPS:
 * wave-cycle section totals; -DMCPT_LANESTATS) write them; slot 63 holds how many work items
 * the last work-item sort of a mesh scene's launch chose to split.  Synchronizes the
 * context's stream.  (Version 2: the n_slots argument; version 1 copied MCPT_DEBUG_SLOTS
 * values, 16 before round 4, whatever the caller's buffer held.) */
int mcpt_debug_counters(mcpt_ctx* ctx, unsigned long long* out, int n_slots, int reset);

/* Copy the local accumulator (n_local_rows × W × 3 f32) to the host and report the
 * number of passes accumulated (the caller divides: fs_frag, montecarlo.cpp:59-70).
 * Synchronizes the context's stream. */
int mcpt_read_accum(mcpt_ctx* ctx, float* rgb_out, int* pass_count);
int mcpt_clear_accum(mcpt_ctx* ctx);
/* The inverse of mcpt_read_accum: load n_local_rows × W × 3 f32 sums and the number of passes
 * they hold into the context's accumulator; later renders add to them (resuming a progressive
 * render from a checkpoint, mcpt_checkpoint_read).  Synchronizes the context's stream. */
int mcpt_write_accum(mcpt_ctx* ctx, const float* rgb, int pass_count);

/* Device pointer of the local accumulator (for an RCCL gather by the caller). */
int mcpt_accum_device_ptr(mcpt_ctx* ctx, void** dev_ptr, size_t* bytes);
/* Device-to-device copy of the local accumulator into a caller buffer of >= bytes
 * (e.g. a torch tensor that feeds the RCCL gather), ordered on the context's stream. */
int mcpt_copy_accum_device(mcpt_ctx* ctx, void* dst_dev_ptr, size_t bytes);

/* Multi-GPU frame assembly inside ONE process (the C++ host's N-GPU path: one context and
 * host thread per device): copy every shard context's local rows into `frame`'s accumulator
 * at their global rows, device to device (hipMemcpyPeerAsync over xGMI, one copy per run of
 * consecutive global rows), ordered after the shards' queued renders and on `frame`'s stream;
 * each shard's stream in turn waits for the copies that read its accumulator, so a
 * progressive caller may render into a shard again right after the call (its next passes
 * cannot reach rows still being copied).
 * `frame` holds a full-frame target of the shards' W x H (mcpt_set_target(W, H, b, 1, 0));
 * rows no shard holds keep their values; every shard must hold the same pass count, which
 * becomes frame's.  Replaces montecarlo.cpp's single-FBO read (:59-70) for sharded renders.
 * Multi-process (torch.distributed) callers gather mcpt_accum_device_ptr with RCCL instead.
 * Asynchronous; mcpt_read_accum(frame) synchronizes. */
int mcpt_gather_rows(mcpt_ctx* frame, mcpt_ctx* const* shards, int n_shards);

/* Select the traversal strategy (mcpt_traversal) for later renders; default AUTO.  AUTO times
 * its schedule candidates on the first launches of >= 2^24 samples after a scene upload — the
 * per-lane walk; the wave-coherent walk (BVH depth < 8 only); the per-lane walk with two and
 * with four pass segments per work item (where the launch has that many segments); for BVH
 * depth >= 8 also the per-lane walk with the deep knobs (leaf batch 16, walk exit 40, min-done 8)
 * at four and at eight segments per item — at most five candidates, each timed twice (forward,
 * then reverse order; each one's best time per sample kept), compared only between launches of
 * the same shape: at most 10 trial launches, run in order on the context's stream (not on the
 * render lanes); a trial's time is read when the call after the next one starts, so AUTO settles
 * two calls after its last trial (mcpt.AUTO_TRIALS = 12 calls).  It never times the stream
 * schedule, which runs only when selected explicitly (MCPT_TRAVERSAL_STREAM).  Later launches of
 * that shape use the fastest — except that, with render lanes on, two segments per item give way
 * to four when the four-segment trials are within 2 % (on the lanes, longer items overlap the
 * previous launch's tail better than the in-order trials show).  mcpt_get_walk_exit /
 * mcpt_get_leaf_batch report the knobs of the
 * candidate the next launch uses.
 * mcpt_get_traversal reports the strategy the next render uses (a trial candidate until AUTO
 * has settled: see mcpt_get_schedule's `settled`).  Every strategy gives the same bits. */
int mcpt_set_traversal(mcpt_ctx* ctx, int mode);
int mcpt_get_traversal(mcpt_ctx* ctx, int* resolved_mode);
/* The whole schedule the next launch of the last launch shape uses: traversal mode, pass
 * segments per work item (MCPT_SEG_PER_ITEM env overrides), and whether AUTO has finished its
 * timing trials (1; always 1 for a fixed mode).  Any pointer may be NULL.  No reference
 * equivalent (the fragment shader has one fixed schedule). */
int mcpt_get_schedule(mcpt_ctx* ctx, int* traversal, int* seg_per_item, int* settled);

/* Per-lane walks (MCPT_TRAVERSAL_LANE): the wave suspends its BVH walk loop once at most
 * `lanes` lanes are still walking, shades the finished lanes and resumes the rest with
 * their next rays (0 = never suspend; -1 = default: 24 with mesh instances, 16 for BVH
 * depth >= 8, else 0).  Same
 * results for every value; a scheduling knob.  mcpt_get_walk_exit reports the value used. */
int mcpt_set_walk_exit(mcpt_ctx* ctx, int lanes);
int mcpt_get_walk_exit(mcpt_ctx* ctx, int* resolved_lanes);

/* Stream schedule (MCPT_TRAVERSAL_STREAM) knobs: path slots (0 = default 16 Mi; never more than
 * the launch's (pixel, pass segment) units; 248 B of device memory per slot, in two pools: 4 GB
 * per context at the default, allocated at the first stream render and freed when
 * mcpt_set_traversal selects another schedule)
 * and the trace kernel's refill threshold (a wave takes new rays for its idle lanes once at
 * most `refill` lanes still walk; 0 = only when all are done; -1 = default 56).  Same results
 * for every value.  mcpt_stream_iterations: trace + shade iterations of the last stream launch
 * (0 if it did not use the stream schedule).  No reference equivalent. */
int mcpt_set_stream_pool(mcpt_ctx* ctx, int slots, int refill);
int mcpt_stream_iterations(mcpt_ctx* ctx, long long* iterations);

/* Per-lane walks: run the primitive-test block only once at least `lanes` lanes wait on a
 * leaf (or no lane can take a node step); others wait (0 = off: node and leaf blocks every
 * iteration; -1 = default: 8 for BVH depth >= 8, else 0).  Same results for every value. */
int mcpt_set_leaf_batch(mcpt_ctx* ctx, int lanes);
int mcpt_get_leaf_batch(mcpt_ctx* ctx, int* resolved_lanes);

/* Render lanes (round 6): once the schedule is settled, the sub-launches of render calls
 * alternate between two internal lanes (HIP streams with their own segment-sum buffers and
 * work-item order state), so a launch's render kernel starts while the previous launch's last
 * workgroups still run; the combines stay in call order on the context's stream, which is
 * ordered after all lane work (results are the same bits).  on = 0: every launch in order on the
 * context's stream.  Default 1 (environment MCPT_OVERLAP=0: 0). */
int mcpt_set_render_lanes(mcpt_ctx* ctx, int on);

/* Bound (bytes) of the device buffer holding the per-chunk partial sums of one launch.  A
 * render call whose pass range spans more 32-pass chunks than fit is run as several launches
 * cut at chunk boundaries (e.g. 84,000 passes at 4K in one call); the accumulator is
 * bit-identical for any budget.  Default 4 GiB (env MCPT_PARTIAL_BYTES at create). */
int mcpt_set_partial_budget(mcpt_ctx* ctx, size_t bytes);
/* (Device memory of a context: the accumulator (12 B per local pixel), the segment sums (up to
 * this budget, allocated by the first launch that needs them) and, with the stream schedule,
 * its pools; the scene buffers.) */
/* Sub-launches the last render call was split into. */
int mcpt_last_launch_count(mcpt_ctx* ctx, int* n_launches);
/* 1 if the last render call ran one pass segment per pass: a call of 2..256 passes whose
 * launch would have fewer than 4 work items per compute unit (e.g. 256x256 at 4 spp) runs each
 * pass as its own segment, so a pixel's passes run side by side, and the combine step sums each
 * 32-pass chunk's passes from 0 in pass order, as one lane would: the bits do not change.
 * Env MCPT_PASS_SPLIT=0/1 forces it off/on. */
int mcpt_last_pass_split(mcpt_ctx* ctx, int* split);

/* Ray queries on the uploaded scene — the shader library calls a TP integrator may use
 * (raytracer_func.frag:718-781, 874-907): traverse_all_bvh (any_hit = 0) or just_hit_bvh
 * (any_hit = 1: stop at the first primitive hit), or with prim >= 0 intersect_one_prim /
 * hit_one_prim (that primitive only), then intersection_info / _color_info / _mat_info.
 * origins, dirs: n × 3 f32 host arrays (directions used as given, like the shader).  A miss
 * has shape = -1, dist = FLT_MAX and zero N/P/colour/material.  Synchronous. */
typedef struct mcpt_hit {
  int shape;          /* primitive type code of the hit (0 mesh, 1 sphere .. 5 quad), -1 = miss */
  int prim;           /* primitive index (after sortEmissiveFirst) */
  int dir;            /* face / part code of the hit (closest_intersection.dir); for a mesh
                         hit the mesh-local triangle index (Mesh_intersect's tri_index) */
  float dist;         /* world distance from the origin */
  float pl[3], pg[3]; /* hit point in primitive space / world space */
  float N[3], P[3];   /* intersection_info: normal and position */
  float color[4];     /* intersection_color_info (rgb, opacity) */
  float material[4];  /* intersection_mat_info (shininess, roughness, emissivity, area) */
} mcpt_hit;
int mcpt_trace(mcpt_ctx* ctx, const float* origins, const float* dirs, int n, int any_hit, int prim,
               mcpt_hit* out);

/* DrawSampling's point cloud (DrawSampling/draw_sampling.cpp:144-150, tp/sampling_base.vert
 * seeding, tp/hsphere.vert random_ray): point k = random_ray(normalize(normal), roughness)
 * with seed floatBitsToUint(fseed) + k * nb_used * (11, 43, 67).  out: n × 3 f32 (host). */
int mcpt_sample_hemisphere(mcpt_ctx* ctx, const float* normal3, const float* fseed3, float roughness,
                           int nb_used, int n, float* out_xyz);

/* Use an external hipStream_t (e.g. torch's current stream); NULL = library stream. */
int mcpt_set_stream(mcpt_ctx* ctx, void* hip_stream);
int mcpt_synchronize(mcpt_ctx* ctx);

/* Device time (ms) of the kernel(s) of the last mcpt_render, from HIP events recorded
 * on the launch stream around the launch.  Synchronizes on the end event. */
int mcpt_last_render_ms(mcpt_ctx* ctx, float* ms);
/* The same interval split into the path-tracing kernel and the chunk-combine kernel
 * (launches spanning more than one 32-pass accumulation chunk). */
int mcpt_last_kernel_ms(mcpt_ctx* ctx, float* trace_ms, float* combine_ms);
/* The same for the render call `back` calls before the last (0: the last).  A context keeps the
 * events of its last 64 calls, so a caller can queue a run of calls and read their times
 * afterwards without waiting after each (waits for that call only). */
int mcpt_kernel_ms_back(mcpt_ctx* ctx, int back, float* trace_ms, float* combine_ms);
/* The path-tracing kernel's whole span (its own start on its stream -> its end), summed over the
 * call's sub-launches, for the call `back` calls before the last (waits for it).  With render lanes
 * (mcpt_set_render_lanes) consecutive launches overlap, and mcpt_kernel_ms_back charges each its
 * period (from the previous launch's render end); the span also counts the overlapped tail, as a
 * profiler's kernel duration does. */
int mcpt_kernel_span_ms_back(mcpt_ctx* ctx, int back, float* span_ms);

/* ---------------------------------------------------------------------------------
 * 2. host scene producer (BVH_GPU_Scene-compatible)
 *    material[7] = { r, g, b, a(opacity), shininess, roughness, emissivity }
 *    (Material, bvh_gpu/scene.h:30-49; Material::light(col,e) = {col, 0, 0, e})
 * --------------------------------------------------------------------------------- */
int mcpt_scene_create(mcpt_scene** out);
int mcpt_scene_destroy(mcpt_scene* s);
int mcpt_scene_clear(mcpt_scene* s);                                            /* gpu_bvh_scene.cpp:76-85 */
int mcpt_scene_add_sphere(mcpt_scene* s, const float* trf16, const float* material7);   /* scene.h:128-133 */
int mcpt_scene_add_cube(mcpt_scene* s, const float* trf16, const float* material7);     /* scene.h:135-142 */
int mcpt_scene_add_cylinder(mcpt_scene* s, const float* trf16, const float* material7); /* scene.h:144-152 */
int mcpt_scene_add_cone(mcpt_scene* s, const float* trf16, const float* material7);     /* scene.h:154-163 */
int mcpt_scene_add_oriented_quad(mcpt_scene* s, const float* trf16, const float* material7); /* scene.h:166-172 */
/* Triangle meshes (BVH_GPU_Scene::add_mesh / place_mesh, gpu_bvh_scene.cpp:51-74,
 * gpu_bvh_scene.h:89-92; ScenePrimitives::add_mesh scene.cpp:56-67).  add_mesh stores a mesh
 * (n_vertices × 3 positions and normals, n_triangles × 3 vertex indices) and builds its own
 * median-split BVH over the triangles (SceneMesh::prim_bb); bb6 = the Mesh::BB() box
 * (min.xyz, max.xyz), NULL = the vertices' bounding box.  place_mesh adds an instance (a
 * CODE_MESH primitive) with transform trf and a material, like the reference. */
int mcpt_scene_add_mesh(mcpt_scene* s, const float* vertices, const float* normals, int n_vertices,
                        const unsigned* tri_indices, int n_triangles, const float* bb6, int* mesh_id);
int mcpt_scene_place_mesh(mcpt_scene* s, int mesh_id, const float* trf16, const float* material7);
/* sizes and flat buffers of all meshes, in the layouts mcpt_upload_meshes takes:
 *   info   : n_meshes × 4 i32 (first node, first leaf, BVH depth, first triangle)
 *   nodes  : n_nodes × 6 f32 (bbmin, bbmax; mesh space)   leaves : n_leaves i32 (triangle or -1)
 *   tris   : n_tris × 3 i32 global vertex ids             verts, normals : n_verts × 3 f32 */
int mcpt_scene_mesh_sizes(mcpt_scene* s, int* n_meshes, int* n_nodes, int* n_leaves, int* n_tris, int* n_verts);
int mcpt_scene_get_mesh_buffers(mcpt_scene* s, int* info, float* nodes, int* leaves, int* tris, float* verts,
                                float* normals);
/* sortEmissiveFirst + BVH_KDtree::compute (scene.cpp:70-88, bvh.cpp:34-93) */
int mcpt_scene_finalize(mcpt_scene* s);
int mcpt_scene_nb_prim(mcpt_scene* s, int* n);
int mcpt_scene_depth(mcpt_scene* s, int* depth);
int mcpt_scene_nb_emissives(mcpt_scene* s, int* n);
/* copy the finalized buffers in the layouts mcpt_upload_scene takes */
int mcpt_scene_get_buffers(mcpt_scene* s, float* prims, float* nodes, int* leaves);
/* overwrite (shininess, roughness, emissivity) and colour of finalized prim i (BVH unchanged;
 * emissivity must keep its sign class: the emissive-first order is fixed at finalize) */
int mcpt_scene_set_material(mcpt_scene* s, int prim, const float* material7);
/* the 8 scene builders of MontecarloGPU/montecarlo.cpp:629-795 (keys Q,W,E,R,T,Y,U,I = 1..8),
 * with light_intensity_ (default 1.2, montecarlo.cpp:138).  Clears, builds, finalizes. */
int mcpt_scene_build_reference(mcpt_scene* s, int scene_id, float light_intensity);

/* canonical camera at aspect W/H: fov 0.78, scene radius 145, frame identity,
 * view = modelview · rotateX(-80); outputs (P·V)^-1 and V^-1, column-major */
int mcpt_camera_canonical(int W, int H, float* invPV16, float* invV16);

/* ---------------------------------------------------------------------------------
 * 3. host helpers: Transfo (easycppogl/gl_eigen.cpp:29-105, degrees, column-major) and
 *    the output step
 * --------------------------------------------------------------------------------- */
int mcpt_transfo_translate(float x, float y, float z, float* out16);           /* Transfo::translate */
int mcpt_transfo_scale(float x, float y, float z, float* out16);               /* Transfo::scale */
int mcpt_transfo_rotate(int axis, float degrees, float* out16);                /* rotateX/Y/Z: axis 0/1/2 */
int mcpt_mat4_mul(const float* a16, const float* b16, float* out16);           /* GLMat4 a * b */
/* fs_frag (montecarlo.cpp:59-70): out = accum / pass_count, per channel */
int mcpt_average(const float* accum, long long n_values, int pass_count, float* out);
/* averaged image (H rows × W × RGB f32, row 0 = bottom) to a little-endian PFM */
int mcpt_write_pfm(const char* path, const float* rgb, int W, int H);
/* what the 8-bit default framebuffer shows: clamp to [0,1], round(255·c), no gamma; PNG RGB8 */
int mcpt_write_png(const char* path, const float* rgb, int W, int H);

/* Checkpoint / resume of a progressive render: the reference's pass loop
 * (montecarlo.cpp:454-466) accumulates into one framebuffer for as long as the window stays
 * open; here a long render (C5: 84,000 passes) can stop and continue in another process with
 * the same bits, because a pass's samples depend only on (pixel, pass, date) and the
 * accumulator is additive.  A file holds the accumulator sums (rows × W × RGB f32, as
 * mcpt_read_accum returns them), the passes they hold, the first pass of the next render call,
 * a caller tag (scene and render parameters) that the reader compares, and the target's
 * identity: the image height H and a hash of the context's image row ids (so a shard's
 * checkpoint cannot be loaded into another shard or another frame of the same local size).
 * Layout, little endian: "MCPTCKP2", int32 W, rows, pass_count, next_pass, tag bytes, H, uint64
 * row-list hash, the tag, then the floats (H = hash = 0: no identity).  The write goes to a
 * temporary file unique to the writer, is flushed to the device (fsync) and renamed over
 * `path`, so an interrupted write or a host crash leaves the previous checkpoint intact.
 * A resumed render equals the uninterrupted one bit for bit when its calls split the pass range
 * at the same points (a call adds its own partial sum of a 32-pass chunk: DESIGN.md §3.3), e.g.
 * the same --chunk in mcpt_render, or call boundaries on multiples of 32 passes. */
#define MCPT_CHECKPOINT_TAG_MAX 1024
/* The context's accumulator, pass count, `next_pass`, `tag` (may be NULL) and target identity.
 * Synchronizes the context's stream. */
int mcpt_checkpoint_save(mcpt_ctx* ctx, const char* path, int next_pass, const char* tag);
/* Resume: loads a file written by mcpt_checkpoint_save for THIS target (W, local rows, H and
 * row ids must match; MCPT_ERR_INVALID_ARG otherwise, and for a file without identity) and,
 * when `tag` is not NULL, with this tag; sets the accumulator and pass count and returns the
 * next call's first pass in *next_pass (may be NULL). */
int mcpt_checkpoint_load(mcpt_ctx* ctx, const char* path, const char* tag, int* next_pass);
/* File-level access without a context (no target identity: H = hash = 0). */
int mcpt_checkpoint_write(const char* path, const float* rgb, int W, int rows, int pass_count, int next_pass,
                          const char* tag);
/* Reads the header into W, rows, pass_count, next_pass (any may be NULL) and the tag into tag_out
 * (MCPT_CHECKPOINT_TAG_MAX bytes, NUL-terminated; may be NULL); the sums into rgb_out
 * (rows × W × 3 floats, at most `capacity` floats) unless it is NULL.  MCPT_ERR_INVALID_ARG for
 * a missing, foreign or truncated file, or sums larger than `capacity`.  Reads "MCPTCKP1" files
 * (round 3, no identity) too. */
int mcpt_checkpoint_read(const char* path, float* rgb_out, long long capacity, int* W, int* rows, int* pass_count,
                         int* next_pass, char* tag_out);

#ifdef __cplusplus
}
#endif

#endif /* MCPT_H_ */
