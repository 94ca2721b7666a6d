// Host/device shared plan structures for one (image size, ORB params) configuration.
// Built once on the host per image size (orbhip_api.cpp::build_plan) and uploaded.
#pragma once
#include <stdint.h>

namespace orbhip {

constexpr int kMaxLevels = 16;
constexpr int kPatchR = 21;                 // 18 (max rotated rBRIEF offset) + 3 (7x7 blur radius)
constexpr int kPatchW = 2 * kPatchR + 1;    // 43
constexpr int kDiscMax = 1024;              // IC_Angle disc offsets (709 for umax of radius 15)

struct LevelGeom {
    int w, h, pitch;
    int64_t pyr_off;          // byte offset of the level inside one frame's pyramid block (level>0)
    float scale;              // mvScaleFactor[l]
    int n_feat;               // mnFeaturesPerLevel[l]
    int min_bx, max_bx, min_by, max_by;   // [16, w-16) x [16, h-16)
    int n_cols, n_rows, w_cell, h_cell;
    int cell_base, n_cells;   // cells of this level in the flat cell table
    int slot_base, n_slots;   // candidate slots of this level (per frame)
    int n_ini;                // DistributeOctTree root count
    float hX;                 // root width
    int kp_cap, kp_base;      // octree output capacity / offset (per frame)
    int rz_noclamp;           // resize taps in [0, 2049] summing to <= 2049: k_resize's saturations are no-ops
    int oct_tab_off;          // octree interval table of the level (u16): max_bx - min_bx column
                              // entries (root << 8 | 6 x-split bits), then max_by - min_by row entries
    int patch_size;           // (int)(31 * scale)
    // resize tables (level l from l-1), offsets into xtab/ytab arrays
    int xtab_off, ytab_off, xmax, vend;
};

struct CellGeom {
    int16_t level, pad;
    int16_t x0, y0;           // window origin in level coordinates (iniX, iniY)
    int16_t wc, hc;           // window size (maxX-iniX, maxY-iniY); 0 when the cell is skipped
    int32_t slot_off;         // first candidate slot (per frame)
};

// k_fast_cells: pair-test survivors kept in LDS per cell. Typically 5-10% of a cell's <= 74 x 74
// pixels pass; a cell with more (noise-like texture) takes the dense path. The cap keeps the
// work-group at ~19 KB of LDS: 8 work-groups (32 waves) per CU at 256 threads, not 5
constexpr int kClistCap = 2048;

struct ExtractPlan {
    int w, h, n_levels;
    int n_cells_total, n_slots_total;   // per frame
    int kp_slots_total;                 // per frame, sum of level kp caps
    int64_t pyr_bytes;                  // per frame (levels 1..L-1)
    int ini_th, min_th;
    int n_disc;
    int blurk[7];                       // bit-exact 7x7 sigma=2 taps, 8 fractional bits
    int max_cells_level;                // max cells of any level (octree LDS carve)
    int clist_cap;                      // FAST survivors listed per cell (<= kClistCap; more -> dense pass)
    int fast_nt;                        // k_fast_cells threads per cell: 0 = by batch size, else 128/256/512/1024
    int fast_win_rows, fast_win_cols;   // largest FAST cell window (<= 50 rows, <= 45 columns: the compact LDS variant)
    LevelGeom lv[kMaxLevels];
};

// Cone pyramid (k_pyr_cone): per (last-level tile, level) the rectangle the tile computes in LDS
// (need, the cone of the levels above) and the part it owns and writes (own). Half-open.
struct ConeRect {
    int16_t nx0, nx1, ny0, ny1;
    int16_t ox0, ox1, oy0, oy1;
};

// Candidate packing: x_rel 12 bits | y_rel 12 bits | score 8 bits (coordinates relative
// to the level's min border, as in vToDistributeKeys).
__host__ __device__ inline uint32_t pack_cand(int x, int y, int score) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}
__host__ __device__ inline int cand_x(uint32_t c) { return (int)(c & 0xFFF); }
__host__ __device__ inline int cand_y(uint32_t c) { return (int)((c >> 12) & 0xFFF); }
__host__ __device__ inline int cand_s(uint32_t c) { return (int)(c >> 24); }

// Octree output record per kept keypoint (level coordinates).
struct LevelKp {
    int16_t x, y;        // level pixel
    uint32_t srl;        // score (8) | inside-lapping-area (1) << 8 | rank among same-flag kps (23) << 9
};

}  // namespace orbhip
