// Shared host/device geometry for the ORB front-end engine (orb_slam3_ros_amd/csrc).
// All per-level constants are derived on the HOST with the reference's exact float/double
// expressions (ORBextractor.cc:409-469, 785-803, 1170-1178) and handed to kernels by value.
#pragma once
#include <stdint.h>

#define ORBFE_MAX_LEVELS 12
#define ORBFE_EDGE 19          // EDGE_THRESHOLD (ORBextractor.cc:73)
#define ORBFE_MINB 16          // EDGE_THRESHOLD - 3 (ORBextractor.cc:789)
#define ORBFE_CELL 35          // W (ORBextractor.cc:785)

struct OrbLevel {
    int w, h;                 // level size (cvRound((float)cols * invScale), ORBextractor.cc:1175)
    int pitch;                // row pitch of this level in the pyramid buffer
    int pyr_off;              // byte offset of the level inside one image's pyramid slab (levels >= 1)
    float scale, inv_scale;   // mvScaleFactor / mvInvScaleFactor
    int patch_size;           // (int)(PATCH_SIZE * scale) (ORBextractor.cc:880)
    // FAST cell grid (ORBextractor.cc:797-803)
    int n_cols, n_rows, w_cell, h_cell;
    int cell_base;            // first global cell index of this level
    int cell_cap;             // max NMS survivors per cell = ceil(wCell/2)*ceil(hCell/2)
    int cellkey_off;          // offset (in keys) of this level's cell slots inside one image
    // octree (ORBextractor.cc:555-579)
    int budget;               // mnFeaturesPerLevel
    int n_ini;                // round((float)(maxX-minX)/(maxY-minY))
    float hx;                 // (float)(maxX-minX)/nIni
    int out_cap;              // max keypoints this level can emit
    int out_off;              // offset of this level in the per-image octree output
    // resize tables (levels >= 1): offsets into the int16 coefficient table
    int tab_x;                // 3*w entries: xofs, alpha0, alpha1
    int tab_y;                // 4*h entries: sy0, sy1 (clipped), beta0, beta1
    int xmax;                 // first dx whose right neighbour leaves the source row
    int simd_end;             // first column handled by the scalar vertical tail
    int rz_rows, rz_cols;     // output rows / cols per k_resize block (fit the LDS source window)
    int rs_ok;                // k_resize_s can build this level (every lane's byte windows fit, host-checked)
    int rs_rows;              // output rows per k_resize_s wave (<= 64)
};

struct OrbGeom {
    int nlevels;
    int width, height;        // level-0 size
    int ini_th, min_th;
    int total_cells;          // cells over all levels
    int cellkeys_per_img;     // key slots over all cells
    int out_per_img;          // octree output slots over all levels
    int kp_cap;               // final keypoints per image (= out_per_img)
    int pyr_bytes;            // bytes of levels >= 1 per image (padded)
    int max_cells_level;      // max cells in one level
    int node_cap;             // octree node capacity (max over levels)
    int pyr_slack;            // offset of a 256 B scratch area at the end of each image's pyramid slab
                              // (k_resize_s's idle lanes store there, so its store count is static)
    OrbLevel lv[ORBFE_MAX_LEVELS];
};

// cv::KeyPoint byte layout (28 B): pt.x, pt.y, size, angle, response, octave, class_id.
struct OrbKeyPoint {
    float x, y, size, angle, response;
    int octave, class_id;
};
