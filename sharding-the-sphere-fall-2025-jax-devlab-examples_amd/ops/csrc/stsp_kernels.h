// Shared declarations of the gfx950 kernels and their C ABI descriptors.
//
// The descriptors are plain C structs mirrored by ctypes (ops/native.py) and
// by the C++ runtime (runtime.cpp).  Pointers are device pointers; scalars are
// carried as double and converted to the kernel's element type at launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// One fused finite-volume RK stage (see stage_kernel.hip).
typedef struct StageDesc {
  const void* X;        // [F][S]  RK combination input, read at own cell (padded layout)
  const void* Q;        // [F][S]  stage input, read with halos (padded layout)
  const void* acc_in;   // [F][S]  RK4 accumulator in (nullable)
  void* out;            // [F][S]
  void* acc_out;        // [F][S]  (nullable)
  const void* recv;     // [R][F]  remote ghost slots (nullable when R == 0)
  const int* gmap;      // [T][4][mg][n]  ghost map (remote slots < 0)
  const int* push;      // [T][4][mg][n]  push map (same-rank ghost slot fed by a strip cell, or -1)
  const int* blocks;    // work list of linear block ids (nullable -> all blocks)
  const void* invA;     // [T][n][n]
  const void* ex;       // [T][n][n+1]  per x-edge coefficient (L, U*L or kappa L/d)
  const void* ey;       // [T][n+1][n]
  const void* mx;       // [T][3][n+1]  x-edge unit normals (SWE)
  const void* my;       // [T][3][n+1]
  const void* cgeo;     // [T][n][n][8] per-cell record (1/A, centre xyz, grad b xyz, 0) (SWE)
  int ntile, n, S, mg, pw;  // pw = n + 2 mg (padded tile width), S = ntile pw^2
  int nblocks;          // number of entries in `blocks` (or total blocks)
  int limiter;
  int remote;           // 1: read remote ghost slots from recv via gmap (boundary blocks)
  double a0, a1, a2, c0, c1, c2, dt;
  double g, omega2;
  void* stamps;         // diagnostic builds only (-DSTSP_STAMPS): [nblocks][16 waves][8] s_memtime per phase
  // ---- direct xGMI halo (xg = 1; see ops/xgmi.py) ----------------------------
  // The producing block stores remote ghost cells straight into the consumer
  // rank's receive ring (IPC-mapped, uncached, STSP_XG_SLOTS slots).  Protocol
  // (stsp_xg_protocol()): 1 = tagged granules, every ghost word travels as an
  // 8-byte {epoch tag, 32-bit payload} atomic store and the consumer re-reads
  // its granules until every tag matches (no counters, no drain); 0 = arrival
  // counters (the producer drains its stores and bumps a counter per peer; a
  // consumer block polls the counters of the peers it reads).
  // `recv` is then this rank's ring base; `push` entries < -1 encode
  // -2 - (peer << 24 | slot).
  int xg;
  int ring;             // per ring slot: elements (counters) or 8-byte granules (tags)
  void* const* peer_ring;                  // [world] ring base of rank p (device array)
  unsigned long long* const* peer_cnt;     // [world] &counter[my rank] on rank p
  const unsigned long long* cnt;           // [world] arrival counters on this rank
  const unsigned long long* nprod;         // [world] producer blocks of rank p feeding this rank
  const int* bmask;     // [nblocks][2] (peers read, peers fed) bit masks
  int* epoch;           // [nblocks] stages completed
  int* err;             // set to 1 on a poll timeout (all later polls fall through)
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  const int* pedge;     // [T] tile sides on a panel edge (bits W, E, S, N); PLR / PPM physics
  // panel-edge ghost interpolation (models/base.py::panel_edge_tables): for tile
  // side s, ghost layer k < 3, strip cell j: ghost = x[b] + t (x[b+1] - x[b]) over
  // the raw strip x of that layer, b = pe_base[t][s][k][j] (tile-local), t = pe_t[...]
  const int* pe_base;   // [T][4][3][n]
  const void* pe_t;     // [T][4][3][n] element type
  // streaming stage only (march_kernel.hip): panel-shared geometry instead of
  // the per-tile records (cgeo, ex, ey), and the topography itself instead of
  // its gradient (ops/hip_compute.py::march_tables)
  const int* torg;      // [T][3] face, I0, J0 of each tile
  const void* crec;     // [Nf*Nf][8] 1/A, S (3), centre (3), 0 in panel-local components (ops/fused.py::kernel_geometry)
  const void* lxt;      // [Nf][Nf+1] x-edge lengths; the y-edge (J', I) has length lxt[I][J']
  const void* bpad;     // [S] topography in the padded layout, ghost ring filled (null: no topography)
  int Nf;               // cells per panel edge
  int frames[6];        // ops/fused.py::frame_code of each panel
  // carried tile-corner ghosts (parallel/layout.py::corner_sources): the strip
  // cells beyond a tile end that the panel-edge interpolation pairs reach.
  // Corner (quad, a, b): quad = (x side E) | 2 (y side N), a rows and b columns
  // beyond the tile corner.
  const int* cgmap;     // [T][4][mg][mg] RankPlan.corner_map: remote slot -1 - m where < 0, else read as stored
  const int* cpush;     // [T][4][mg][mg] slot fed by the own cell of corner block (quad, a, b): >= 0 same
                        // rank, < -1 remote code (as push), -1 none (nullable)
} StageDesc;

int stsp_stage_launch(int phys, int dtype, int bx, int by, const StageDesc* d, hipStream_t stream);
// Pipelined streaming SSP-RK3 step (march3_kernel.hip): one launch marches all
// three stages up each strip of a tile (stage s + 1 trails stage s by two rows),
// reading the step input d->Q once and writing the step output d->out at the
// cells at least 4 from a tile edge.  Stage s computes out = b0[s] X + b1[s] Q
// + b2[s] dt L(Q) with X = the step input.  The cells within D of a tile edge of
// the stage-1 and stage-2 results go to q1 / q2 (stage 1 also pushes its
// same-rank ghost copies into q1), so that two band launches of the stage kernel
// finish stages 2 and 3 next to the tile edges (ops/march3.py).
typedef struct March3Desc {
  void* q1;
  void* q2;
  double b0[3], b1[3], b2[3];
  int D;
} March3Desc;
int stsp_march3_launch(int dtype, int rows, const StageDesc* d, const March3Desc* m, hipStream_t stream);
int stsp_pack_launch(int dtype, const void* q, int S, int F, const int* idx, int ns, void* send, hipStream_t stream);
int stsp_copy_index_launch(int dtype, const void* src, const int* sidx, void* dst, const int* didx, int k,
                           int batch, long src_stride, long dst_stride, hipStream_t stream);
// Direct xGMI halo: write the remote ghost cells of state q (entries src[i] ->
// code[i] = peer << 24 | slot) into every peer's ring slot of stage `epoch`.
int stsp_xg_prime_launch(int dtype, const void* q, int S, int F, const int* src, const int* code, int nent,
                         void* const* peer_ring, int ring, int epoch, hipStream_t stream);
// One fused SSP-RK3 step of the shallow-water solver (fused_step.hip, ops/fused.py):
// temporal blocking over a window of the block plus a ring of 2 NS cells.
typedef struct FusedDesc {
  const void* Q;        // [F][S] step input, padded layout
  void* out;            // [F][S] step output: interior + same-rank ghost pushes
  const int* src;       // [nb][W*W] padded offset of each window cell's source, -1 = not loaded
  const int* org;       // [nb][4] X0, Y0, tile_local, xo | yo << 12 | region flags << 24 | face << 29
  // geometry (ops/fused.py::kernel_geometry): panel-independent tables, no
  // per-cell records; blocks with a side region also read their own face
  // lengths and line normals
  const void* len;      // [nb][2 H1 (H1+1)] x-faces, then y-faces
  const void* nrm;      // [nb][2][5][3][W+1] line normals per region, component-major
  const void* tane;     // [N+1]
  const void* crec;     // [N*N][8] 1/A, S (3), centre (3), 0 in panel-local components
  const void* lxt;      // [N][N+1]
  const void* gbt;      // [S (+ ring)][4] grad b, padded layout; null without topography
  int frames[6];
  const void* code;     // [nb][W*W] u64: 4 x int16 neighbour codes per window cell and side (-1, entry, -3)
  const int* gtab;      // [nb][G][2] LDS index of the interpolation pair
  const void* gw;       // [nb][G] interpolation weights
  const int* ctab;      // [nb][C][16] corner faces (ops/fused.py::corner_tables): per side q (c, d) the cell's
                        // LDS index and its across / inward stencil pairs (5 ints), face slots c, d, flags
  const void* cgf;      // [nb][C][8] normal out of c, length, the four stencil weights
  const int* ccnt;      // [nb]
  const int* push;      // [T][4][mg][n] push map (same-rank ghost slot fed by a strip cell, or -1)
  int G, C;
  int nblocks, n, N, S, mg, pw;
  int B, ns, limiter;
  double a0[4], a1[4], a2[4];
  double dt, g, omega2;
  // several ranks (xg = 1, ops/fused.py::FusedExchangePlan): window cells with
  // src <= -2 are read from this rank's receive ring, slot epoch % STSP_XG_SLOTS,
  // entry -2 - src, as tagged granules; every step stores the block's cells that
  // peers read into their rings (xpush codes peer << 24 | entry), tag epoch + 2
  int xg;
  int ring;                 // 8-byte granules per ring slot
  const void* recv;         // this rank's ring (granules)
  void* const* peer_ring;   // [world] ring bases (IPC-mapped)
  const int* xpush;         // [nb][B*B][K] destination codes, -1 none
  int K;
  int* epoch;               // [nb] steps completed
  int* err;                 // set to 1 on a wait timeout (every later wait falls through)
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  // nullable: [nb][16 waves][16] s_memtime of every wave at the phase boundaries
  // (prologue, then faces / updates of each stage, end); profiling only
  unsigned long long* stamps;
  // one rank holding every tile in id order: the kernel computes each window
  // cell's storage offset from the cube topology (links: per face, sides W E S
  // N, 6 bits each: nbr face | nbr edge << 3 | reversed << 5) instead of
  // loading `src` (one dependent memory round trip less in the prologue)
  int local_src;
  int links[6];
  // several steps per launch (0 / 1 = one): needs every block co-resident
  // (checked by the launcher), epoch / err, and prod [nb][PM] (producer blocks of
  // each block's window, -1 padded, symmetric)
  int nsteps;
  const int* prod;
  int PM;
  const int* cpush;     // [T][4][mg][mg] carried corner ghost pushes (StageDesc::cpush), nullable
  // face-pass schedule (ops/fused.py::pass_schedule): [nb][3 stages][17] u32:
  // per wave (16) bit p set = the wave runs pass p (faces 64 p .. 64 p + 63) of
  // the stage, balanced over the CU's four SIMDs (waves w and w + 4 share one);
  // word 16 bit p = pass p holds a face next to a panel-edge line
  const unsigned* sched;
  const void* nrmf;     // [nb][3][2 H1 (H1+1)] per-face normals of panel-edge blocks (component-major)
  // tagged in-launch hand-off of a multi-step launch, [2][W][S] u64 (W = 5 fp64, 4 fp32)
  // zero-initialised and kept with the epoch array; null = epoch hand-off
  void* hx;
  // per-cell producer polls of a one-rank epoch hand-off: [nb][W*W] int8
  // index into prod[b] of the producer of each window cell (-1: none); null =
  // wave 0 polls every producer before a barrier
  const signed char* pidx;
} FusedDesc;
int stsp_fused_launch(int dtype, const FusedDesc* d, hipStream_t stream);
int stsp_fused_limits(int* gmax, int* cmax);
int stsp_fused_tagh(void);
// the fused step's packed cell records (granules per cell) and their initial
// delivery into the peers' xGMI rings
int stsp_fused_record_words(int dtype);
int stsp_fused_prime_launch(int dtype, const void* q, int S, const int* src, const int* code, int nent,
                            void* const* peer_ring, int ring, int epoch, hipStream_t stream);
// Direct xGMI halo build constants: protocol (0 counters, 1 tagged granules), ring slots.
int stsp_xg_protocol(void);
int stsp_xg_slots(void);
}
