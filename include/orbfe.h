/*
 * orbfe.h — C-ABI of the MI355X-native ORB front-end (liborbfe.so).
 *
 * Drop-in boundary for the Tracking-thread hot path of ORB-SLAM3 as vendored in
 * giltchcity/orb_slam3_ros. Every entry point names the reference interface it replaces
 * (paths under orb_slam3/). Plain pointers and sizes only; no exceptions cross the ABI; every
 * call returns an int status (>= 0 ok, see ORBFE_E_*). Handles are not re-entrant (like one
 * ORBextractor instance, whose mvImagePyramid is per-call state); distinct handles may be used
 * concurrently from different host threads. Matcher entry points are stateless and re-entrant.
 *
 * Keypoints use the 28-byte cv::KeyPoint layout (pt.x, pt.y, size, angle, response, octave,
 * class_id) so a shim can memcpy them into std::vector<cv::KeyPoint>; descriptors are n x 32 u8
 * rows (cv::Mat CV_8U, continuous).
 */
#ifndef ORBFE_H
#define ORBFE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBFE_OK 0
#define ORBFE_E_EMPTY (-1)      /* empty image: ORBextractor::operator() returns -1 (ORBextractor.cc:1090-1091) */
#define ORBFE_E_ARG (-2)        /* bad type / size / argument (the reference asserts CV_8UC1, :1094) */
#define ORBFE_E_DEVICE (-3)     /* HIP runtime error */
#define ORBFE_E_CAPACITY (-4)   /* caller buffer too small */

typedef struct orbfe_keypoint {  /* == cv::KeyPoint */
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbfe_keypoint;

typedef struct orbfe_extractor orbfe_extractor;

/* ---------------------------------------------------------------------------------------------
 * Extractor — replaces ORB_SLAM3::ORBextractor (include/ORBextractor.h:43-112)
 * ------------------------------------------------------------------------------------------- */

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * (ORBextractor.h:49-50, ORBextractor.cc:409-469). Binds to the current HIP device. */
int orbfe_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                           orbfe_extractor** out);
void orbfe_extractor_destroy(orbfe_extractor* h);

/* GetLevels / GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (ORBextractor.h:61-81). Arrays have nlevels entries; any may be NULL.
 * features_per_level: mnFeaturesPerLevel (ORBextractor.cc:434-445). */
int orbfe_extractor_levels(const orbfe_extractor* h);
int orbfe_extractor_scale_info(const orbfe_extractor* h, float* scale, float* inv_scale, float* sigma2,
                               float* inv_sigma2, int* features_per_level);

/* OpenCV-behaviour model of the two OpenCV primitives whose 8-bit results depend on how the
 * OpenCV the reference links was built (the reference itself cannot be built here):
 *   resize_simd_lanes: cv::resize INTER_LINEAR (ORBextractor.cc:1183). Columns covered by the
 *     universal-intrinsic vertical pass (VResizeLinearVec_32s8u: blocks of `lanes` u8, then of
 *     lanes/2) round as ((((H0>>4)*b0)>>16) + (((H1>>4)*b1)>>16) + 2) >> 2, the rest with the
 *     scalar (H0*b0 + H1*b1 + 2^21) >> 22. 16 = SSE2/NEON baseline (default), 32 = AVX2, 64 =
 *     AVX-512 (CV_SIMD256 / 512 builds), 8 = a half-width build, 0 = no SIMD (scalar only).
 *   blur_variant: cv::GaussianBlur 7x7 sigma 2 8U (ORBextractor.cc:1133) Q8 kernel quantisation;
 *     0 = error-diffusion [18,34,48,56,48,34,18] (OpenCV >= 3.4.6, default), 1 = per-tap rounding
 *     [18,34,49,55,49,34,18] (older builds).
 * Other values return ORBFE_E_ARG. Changing the model waits for the device, releases the handle's
 * batch buffers (the last batch's outputs and pyramid are gone) and rebuilds them on the next call. */
int orbfe_extractor_set_opencv_model(orbfe_extractor* h, int resize_simd_lanes, int blur_variant);
int orbfe_extractor_get_opencv_model(const orbfe_extractor* h, int* resize_simd_lanes, int* blur_variant);

/* Max keypoints one image can yield (sum over levels of the octree bound); size caller buffers with it. */
int orbfe_extractor_capacity(orbfe_extractor* h, int width, int height);

/* int ORBextractor::operator()(InputArray image, InputArray mask, vector<KeyPoint>& kps,
 *                              OutputArray desc, vector<int>& vLappingArea)   (ORBextractor.h:57-59)
 * Host buffers: img is width x height u8 with row stride `stride` bytes. The mask is ignored, as in
 * the reference. lap0/lap1 = vLappingArea[0..1]. On success returns monoIndex (>= 0) and writes
 * *n keypoints / descriptors; returns ORBFE_E_EMPTY for an empty image.
 * Per call: one pinned upload, the handle's launches, one result copy, one synchronisation. */
int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int width, int height, int stride, int lap0, int lap1,
                  orbfe_keypoint* kps, uint8_t* desc, int cap, int* n);

/* The public std::vector<cv::Mat> mvImagePyramid (ORBextractor.h:83), read by
 * Frame::ComputeStereoMatches (Frame.cc:818,908,918,923): copies level `level` of image `image`
 * of the last call to dst (row pitch dst_pitch) and reports its size. dst may be NULL. */
int orbfe_pyramid_level(orbfe_extractor* h, int image, int level, uint8_t* dst, int dst_pitch, int* width,
                        int* height);

/* Batched device path (multi-camera / multi-frame; Frame.cc:122-125 runs two extractors on two
 * threads per stereo frame — here one launch sequence covers nimg images). d_imgs: nimg device
 * pointers (host array) to width x height u8 images with row pitch `pitch`; each image must have
 * pitch * height readable bytes (the level-1 build reads whole 12-byte windows of the last row, past
 * the width when pitch > width; a view into a larger frame satisfies this). stream: hipStream_t
 * (NULL = the legacy default stream, as for every stream argument here). Outputs stay on the device:
 * see orbfe_batch_outputs. */
int orbfe_extract_batch(orbfe_extractor* h, int nimg, const uint8_t* const* d_imgs, int width, int height,
                        int pitch, int lap0, int lap1, void* stream);
/* orbfe_extract_batch with a vLappingArea per image: laps[2*i], laps[2*i+1] (host array) for image i,
 * e.g. the left and right KannalaBrandt8 cameras' own mvLappingArea (Frame.cc:1059-1060). */
int orbfe_extract_batch_laps(orbfe_extractor* h, int nimg, const uint8_t* const* d_imgs, int width, int height,
                             int pitch, const int32_t* laps, void* stream);

/* Device pointers of the last batch: kps[nimg][cap], desc[nimg][cap][32], counts[nimg][2] =
 * {n, monoIndex}. Valid until the next call on this handle. */
int orbfe_batch_outputs(orbfe_extractor* h, orbfe_keypoint** d_kps, uint8_t** d_desc, int** d_counts, int* cap);

/* Make later orbfe_extract_batch calls write their outputs into caller-owned device buffers
 * (kps[cap_images][cap], desc[cap_images][cap][32], counts[cap_images][2]) instead of the
 * handle's own; cap = orbfe_extractor_capacity(). Pass NULLs to revert. While bound, a batch of more
 * than cap_images images fails with ORBFE_E_CAPACITY. The host API (orbfe_extract) never uses them. */
int orbfe_set_batch_outputs(orbfe_extractor* h, orbfe_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                            int cap_images);

/* Per-kernel HIP-event timing (for bench.py's roofline). While enabled, every batch records
 * events around each stage on the stream it runs on (no host sync). orbfe_get_stage_timing waits
 * for the recorded batches, writes the MEAN ms per batch of each stage to ms[0..ORBFE_NUM_STAGES)
 * = {pyramid + FAST (all levels), octree, describe}, resets, and returns the batch count. */
#define ORBFE_NUM_STAGES 3
int orbfe_set_stage_timing(orbfe_extractor* h, int enable);
int orbfe_get_stage_timing(orbfe_extractor* h, float* ms);
/* While stage timing is enabled, the host-API calls time themselves with HIP events on their stream:
 * ms[0..2] = the last orbfe_extract's {image upload, kernels, result copies (count read-back and
 * keypoint / descriptor copies)}, ms[3..4] = the last orbfe_stereo_match with h as the left handle
 * {kernels, result copies}. Returns 5 (0 when timing is off: ms then holds the last timed values). */
int orbfe_get_call_timing(orbfe_extractor* h, float* ms);

/* ---------------------------------------------------------------------------------------------
 * Stereo — replaces Frame::ComputeStereoMatches (include/Frame.h:116, src/Frame.cc:811-981)
 * ------------------------------------------------------------------------------------------- */

/* Rectified pinhole stereo for nframes frames: frame f's left image is image (lbase + f*lstep) of
 * the last batch of `left`, its right image is image (rbase + f*rstep) of the last batch of
 * `right` (left == right allowed, e.g. interleaved L/R). bf = mbf, fx = K(0,0) (the reference
 * reads mb = mbf/fx). Device outputs: uright/depth[nframes][cap] (-1 = no match, Frame.cc:813-814),
 * nmatch[nframes] (matches before the median cut). */
int orbfe_stereo_match_batch(orbfe_extractor* left, int lbase, int lstep, orbfe_extractor* right, int rbase,
                             int rstep, int nframes, float bf, float fx, float* d_uright, float* d_depth,
                             int* d_nmatch, void* stream);

/* Host convenience for one frame: uses the last orbfe_extract call of `left` and `right` and writes
 * host arrays uright[n_left], depth[n_left]. Returns the pre-cut match count. */
int orbfe_stereo_match(orbfe_extractor* left, orbfe_extractor* right, float bf, float fx, float* uright,
                       float* depth);

/* Frame::Frame(stereo) (src/Frame.cc:101-141) in one call: ExtractORB(0, imLeft) and ExtractORB(1,
 * imRight) (:122-125, ORBextractor::operator() with vLappingArea {0, 0}), then ComputeStereoMatches
 * (:141), with host images in and host results out. Replaces the two per-frame std::threads plus
 * orbfe_extract x 2 + orbfe_stereo_match: both images go up in one pinned copy, run as ONE two-image
 * batch on `left` (image 0 = left, image 1 = right: orbfe_pyramid_level(left, 1, ...) is the right
 * extractor's mvImagePyramid afterwards) with the stereo kernels on the same stream, and every result
 * comes back before one synchronisation. `right` must have left's parameters (Tracking builds both
 * extractors from the same settings, Tracking.cc:637-645; else ORBFE_E_ARG); it is not written.
 * Outputs as orbfe_extract for each side (n_*, mono_* = monoIndex) and orbfe_stereo_match
 * (uright / depth [n_left]). Returns the pre-cut stereo match count. orbfe_get_call_timing(left)
 * then holds {upload, extraction kernels, result copies, stereo kernels, 0}; the upload slot runs
 * from the left image's push to the right image's, so it includes the right image's host packing. */
int orbfe_frame_stereo(orbfe_extractor* left, orbfe_extractor* right, const uint8_t* img_left,
                       const uint8_t* img_right, int width, int height, int stride, float bf, float fx,
                       orbfe_keypoint* kps_left, uint8_t* desc_left, int cap_left, int* n_left, int* mono_left,
                       orbfe_keypoint* kps_right, uint8_t* desc_right, int cap_right, int* n_right,
                       int* mono_right, float* uright, float* depth);

/* Frame::Frame(imLeft, imRight, ..., KannalaBrandt8 rig) (src/Frame.cc:1034-1105) up to its descriptor
 * matching, in one call like orbfe_frame_stereo: ExtractORB(0, imLeft) and ExtractORB(1, imRight)
 * with vLappingArea {lap0, lap1} (:1059-1062; TUM-VI overlappingBegin/End), then
 * ComputeStereoFishEyeMatches' knnMatch(k = 2) + ratio test of the lapping rows (:1126-1151), as ONE
 * two-image launch chain on `left`. l2r[n_left]: the right keypoint index (mvKeysRight numbering) of
 * each left keypoint whose ratio test passes, -1 otherwise (the mvLeftToRightMatch candidates that
 * the camera model's TriangulateMatches then confirms on the host, :1152-1160); dist[n_left] their
 * Hamming distance or -1. Returns the passing query count (the kNN stage's good matches). */
int orbfe_frame_fisheye(orbfe_extractor* left, orbfe_extractor* right, const uint8_t* img_left,
                        const uint8_t* img_right, int width, int height, int stride, int lap0, int lap1, float ratio,
                        orbfe_keypoint* kps_left, uint8_t* desc_left, int cap_left, int* n_left, int* mono_left,
                        orbfe_keypoint* kps_right, uint8_t* desc_right, int cap_right, int* n_right,
                        int* mono_right, int32_t* l2r, int32_t* dist);

/* ---------------------------------------------------------------------------------------------
 * ORBmatcher — replaces the Tracking-thread methods of ORB_SLAM3::ORBmatcher (include/ORBmatcher.h)
 * and Frame::ComputeStereoFishEyeMatches' brute-force kNN. Stateless and re-entrant; every call
 * takes host pointers, runs on the current HIP device, and returns nmatches (>= 0) or an error.
 * The C++ objects the reference passes (Frame&, KeyFrame*, MapPoint*, FeatureVector) are
 * flattened by the caller into the snapshot structs below under the objects' own locks
 * (MapPoint::GetDescriptor / isBad / Observations, MapPoint.cc:210,302,405); MapPoint* results
 * are returned as the caller's int32 handles (-1 = NULL).
 * ------------------------------------------------------------------------------------------- */
int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b);   /* DescriptorDistance (ORBmatcher.cc:2058-2074) */

#define ORBFE_GRID_COLS 64   /* FRAME_GRID_COLS (Frame.h:44) */
#define ORBFE_GRID_ROWS 48   /* FRAME_GRID_ROWS (Frame.h:45) */

/* The parts of a Frame the matchers read (Frame.h). Keypoints are mvKeysUn (== mvKeys for the
 * rectified / undistorted case); the 64x48 grid (AssignFeaturesToGrid, Frame.cc:385-416) is
 * rebuilt from them with the reference's PosInGrid arithmetic.
 * Two-camera frames (Nleft != -1: the KannalaBrandt8 stereo constructor, Frame.cc:1000-1125):
 * two_cams = 1, keys = mvKeys [0, nleft) followed by mvKeysRight [nleft, n) (the reference's
 * AssignFeaturesToGrid reads exactly these, Frame.cc:401-403), desc / mvpMapPoints rows in the same
 * numbering (mDescriptors = [left; right]), a left grid over [0, nleft) and a right grid (mGridRight)
 * over [nleft, n); l2r / r2l = mvLeftToRightMatch / mvRightToLeftMatch. A zero-initialised tail
 * (two_cams = 0) is the single-camera frame (Nleft == -1). */
typedef struct orbfe_frame {
    int32_t n;                       /* N */
    const orbfe_keypoint* keys;      /* mvKeysUn [n] (two_cams: mvKeys ++ mvKeysRight) */
    const uint8_t* desc;             /* mDescriptors [n][32] */
    const float* uright;             /* mvuRight [n] or NULL (monocular; not read for two_cams) */
    float min_x, max_x, min_y, max_y;   /* mnMinX, mnMaxX, mnMinY, mnMaxY (ComputeImageBounds) */
    int32_t nlevels;
    const float* scale_factors;      /* mvScaleFactors [nlevels] */
    float mbf;                       /* mbf (stereo baseline * fx) */
    int32_t two_cams;                /* 1: Nleft != -1 (fields below valid) */
    int32_t nleft;                   /* Nleft, 0 <= nleft <= n */
    const int32_t* l2r;              /* mvLeftToRightMatch [nleft] (right index or -1) */
    const int32_t* r2l;              /* mvRightToLeftMatch [n - nleft] (left index or -1) */
    int32_t device;                  /* 1: keys / desc / uright / scale_factors are device pointers
                                        (orbfe_frame_device_view); 0: host memory */
} orbfe_frame;

/* The current frame kept on the device for Tracking's searches. orbfe_extractor_frame_id(h) counts
 * h's extractions; read it right after orbfe_frame_stereo (the shim keeps it in the Frame).
 * orbfe_frame_device_view(left, id, F) then fills F with the DEVICE view of that call's left image
 * (mvKeysUn / mDescriptors / mvuRight of the pinhole stereo Frame, Frame.cc:101-141): n, keys, desc,
 * uright, nlevels, scale_factors, device = 1 (the caller sets the bounds and mbf as for a host view).
 * ORBFE_E_ARG when h has extracted since (the view would show another frame). The host-API
 * single-camera searches (orbfe_search_by_projection_local / _lastframe / _kf,
 * orbfe_search_local_points(_track)) take such a view for frames of <= 2048 keypoints and <= 2048
 * queries and read the frame from HBM instead of the caller's copy (no per-call upload of ~64 KB);
 * other shapes return ORBFE_E_ARG (pass the host view). Valid until h's next extraction. */
uint64_t orbfe_extractor_frame_id(orbfe_extractor* h);
int orbfe_frame_device_view(orbfe_extractor* left, uint64_t frame_id, orbfe_frame* F);

/* MapPoint tracking snapshot for SearchByProjection(Frame&, vector<MapPoint*>, ...)
 * (MapPoint.h:172-180; filled by Frame::isInFrustum, Tracking.cc:3407-3425). 80 bytes. */
#define ORBFE_MP_IN_VIEW 1           /* mbTrackInView */
#define ORBFE_MP_BAD 2               /* isBad() */
#define ORBFE_MP_IN_VIEW_R 8         /* mbTrackInViewR (two-camera frames, Frame.cc:575-584) */
typedef struct orbfe_map_point {
    float proj_x, proj_y, proj_xr;   /* mTrackProjX, mTrackProjY, mTrackProjXR (two_cams: the right-camera x) */
    float view_cos;                  /* mTrackViewCos */
    float depth;                     /* mTrackDepth */
    int32_t scale_level;             /* mnTrackScaleLevel */
    int32_t flags;                   /* ORBFE_MP_* */
    int32_t observations;            /* Observations() */
    int32_t id;                      /* handle stored into mvpMapPoints */
    float proj_yr;                   /* mTrackProjYR (two-camera frames, Frame.cc:1227-1230) */
    float view_cos_r;                /* mTrackViewCosR */
    int32_t scale_level_r;           /* mnTrackScaleLevelR (-1: right branch skipped) */
    uint8_t desc[32];                /* GetDescriptor() */
} orbfe_map_point;

/* ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints)
 * (ORBmatcher.cc:43-213). mvp: F.mvpMapPoints as handles [F.n], updated in place; mvp_obs:
 * Observations() of the MapPoint currently in each slot (0 when empty). Points are processed in
 * array order exactly as the reference loop (a keypoint already holding a point with
 * Observations() > 0 is skipped). Two-camera frames (F->two_cams) take the reference's Nleft != -1
 * branches: the left search without the mvuRight check, the stereo partner slot written through
 * mvLeftToRightMatch (:124-128), and the right-camera search over the right grid with the
 * ORBFE_MP_IN_VIEW_R fields (:138-209: radius NOT scaled by th, partner through
 * mvRightToLeftMatch). Returns nmatches. */
int orbfe_search_by_projection_local(const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs,
                                     const orbfe_map_point* mps, int32_t n_mps, float th, int32_t bFarPoints,
                                     float thFarPoints, float nnratio);

/* Device-resident forms for pipelines that keep frames and map points in HBM: F's keys / desc /
 * uright / scale_factors, d_mvp, d_mvp_obs and the records are DEVICE pointers written on `stream`
 * (hipStream_t, NULL = legacy default); the matcher waits for that stream, writes d_mvp in place
 * and returns nmatches once the results are complete. Semantics are those of the host forms;
 * records with a scale level outside [0, nlevels) are skipped (the host forms reject them). */
int orbfe_search_by_projection_local_device(const orbfe_frame* F, int32_t* d_mvp, const int32_t* d_mvp_obs,
                                            const orbfe_map_point* d_mps, int32_t n_mps, float th,
                                            int32_t bFarPoints, float thFarPoints, float nnratio, void* stream);

/* One projected point of the last frame for SearchByProjection(CurrentFrame, LastFrame, th, bMono)
 * (ORBmatcher.cc:1676-1887): the caller projects LastFrame.mvpMapPoints[i] with Tcw
 * (x3Dc = Tcw * X, invzc = 1/z, uv = K * x3Dc) and skips outliers / empty slots (valid = 0). */
typedef struct orbfe_proj_point {
    float u, v, invzc;
    int32_t octave;                  /* LastFrame keypoint octave (nLastOctave) */
    float angle;                     /* LastFrame keypoint angle (rotation histogram) */
    int32_t valid;
    int32_t observations;            /* Observations() of the MapPoint */
    int32_t id;                      /* MapPoint handle */
    uint8_t desc[32];
} orbfe_proj_point;                  /* 64 bytes */

/* Motion-model search: bForward / bBackward as computed by the reference from the poses
 * (ORBmatcher.cc:1691-1693). Returns nmatches after the rotation-consistency filter. */
int orbfe_search_by_projection_lastframe(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                         const orbfe_proj_point* pts, int32_t n_pts, float th, int32_t bForward,
                                         int32_t bBackward, int32_t checkOri);

/* The same search for a two-camera CurrentFrame (CurrentFrame.Nleft != -1, ORBmatcher.cc:1794-1858):
 * right_uv[2 i] / right_uv[2 i + 1] = mpCamera->project(GetRelativePoseTrl() * x3Dc) of point i (the
 * caller's camera model); after the left search (left grid, no mvuRight check; a point whose left
 * window is empty skips both, :1738-1739) the right grid is searched and the slot nleft + bestIdx2
 * written; both enter the rotation histogram. pts[i].octave is nLastOctave (LastFrame.mvKeys /
 * mvKeysRight). For a single-camera cur (two_cams = 0) right_uv is ignored (== the function above). */
int orbfe_search_by_projection_lastframe_stereo(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                                const orbfe_proj_point* pts, const float* right_uv, int32_t n_pts,
                                                float th, int32_t bForward, int32_t bBackward, int32_t checkOri);

/* Relocalisation refinement SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
 * (ORBmatcher.cc:1889-2010): one entry per KF map point that is not bad and not already found,
 * projected by the caller; octave = PredictScale(...) (MapPoint.cc:531-546), angle =
 * pKF->mvKeysUn[i].angle; valid = 0 when the reference's bounds / distance checks reject it.
 * Any slot already holding a MapPoint is skipped. */
int orbfe_search_by_projection_kf(const orbfe_frame* cur, int32_t* mvp, const orbfe_proj_point* pts,
                                  int32_t n_pts, float th, int32_t ORBdist, int32_t checkOri);

/* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:648-763).
 * prev_matched: [F1.n][2] (x, y), updated in place; matches12: [F1.n] output. */
int orbfe_search_for_initialization(const orbfe_frame* F1, const orbfe_frame* F2, float* prev_matched,
                                    int32_t* matches12, int32_t windowSize, float nnratio, int32_t checkOri);

/* DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) flattened: node ids ascending,
 * offsets[n_nodes + 1] into indices. */
typedef struct orbfe_feature_vector {
    int32_t n_nodes;
    const uint32_t* node_ids;
    const int32_t* offsets;
    const uint32_t* indices;
} orbfe_feature_vector;

/* SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:223-425).
 * kf_mp: pKF->GetMapPointMatches() handles with bad points already mapped to -1; out: [F.n].
 * kf_keys[i] is the keypoint the reference reads for KF index i (mvKeysUn, or for a two-camera KF
 * mvKeys / mvKeysRight by side, :327-329). A two-camera F (F->two_cams) takes the Nleft != -1 walk:
 * separate left / right best-and-second, the right match only inside the left's bestDist1 <= TH_LOW
 * and its ratio test disabled (the reference's "|| true", :359). */
int orbfe_search_by_bow(const orbfe_keypoint* kf_keys, const uint8_t* kf_desc, const int32_t* kf_mp, int32_t kf_n,
                        const orbfe_feature_vector* kf_fv, const orbfe_frame* F, const orbfe_feature_vector* f_fv,
                        int32_t* out, float nnratio, int32_t checkOri);

/* ComputeStereoFishEyeMatches' descriptor stage (Frame.cc:1126-1151): BFMatcher(NORM_HAMMING)
 * knnMatch(k=2) of left rows [0, nl) against right rows [0, nr) and Lowe's 0.7 ratio. out_train[i]
 * = best right row of left row i or -1; out_dist[i] its distance. The KannalaBrandt8
 * TriangulateMatches post-filter stays with the camera model on the host. */
int orbfe_stereo_knn_ratio(const uint8_t* left_desc, int32_t nl, const uint8_t* right_desc, int32_t nr,
                           float ratio, int32_t* out_train, int32_t* out_dist);

/* Batched, device-resident form of the same stage for nframes KannalaBrandt8 stereo frames over
 * the last batch outputs of the extractor handles (the lapping-area rows the reference slices out,
 * Frame.cc:1129-1133): frame f's queries are rows [monoIndex, n) of left image (lbase + f*lstep),
 * its train rows [monoIndex, n) of right image (rbase + f*rstep) (left == right allowed).
 * Device outputs, [nframes][cap] in the frame's full keypoint numbering: d_l2r[i] = right keypoint
 * index (trainIdx + monoRight) if Lowe's test passes (the mvLeftToRightMatch candidate before the
 * host-side TriangulateMatches depth check) else -1; d_dist[i] its distance or -1;
 * d_ngood[nframes] = passing queries per frame (descMatches). Enqueued on stream, no host sync. */
int orbfe_stereo_knn_batch(orbfe_extractor* left, int lbase, int lstep, orbfe_extractor* right, int rbase, int rstep,
                           int nframes, float ratio, int32_t* d_l2r, int32_t* d_dist, int32_t* d_ngood, void* stream);

/* The same stage over explicit device output blocks instead of extractor handles: the layout of
 * orbfe_batch_outputs / orbfe_set_batch_outputs (counts [image][2] = {n, monoIndex}, descriptors
 * [image][cap][32]), e.g. the slots an all-gather brought from the rank that extracted the other
 * camera (BASELINE config 4 over several GPUs: the left and right image of a stream on two ranks,
 * SURVEY.md §8(e)). Frame f pairs left image (lbase + f*lstep) with right image (rbase + f*rstep).
 * Outputs and stream as orbfe_stereo_knn_batch. */
int orbfe_stereo_knn_slabs(const int32_t* d_counts_l, const uint8_t* d_desc_l, int lbase, int lstep,
                           const int32_t* d_counts_r, const uint8_t* d_desc_r, int rbase, int rstep, int cap,
                           int nframes, float ratio, int32_t* d_l2r, int32_t* d_dist, int32_t* d_ngood, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Local-map projection (the step before SearchByProjection in Tracking::SearchLocalPoints,
 * Tracking.cc:3407-3452): Frame::isInFrustum (pinhole branch, Frame.cc:512-570) and
 * MapPoint::PredictScale (MapPoint.cc:531-546) for every local map point, on the device.
 * ------------------------------------------------------------------------------------------- */
#define ORBFE_MP_SKIP 4              /* mnLastFrameSeen == current frame id: not projected */
typedef struct orbfe_map_point_3d {
    float pos[3];                    /* GetWorldPos() */
    float normal[3];                 /* GetNormal() */
    float min_dist, max_dist;        /* mfMinDistance, mfMaxDistance (GetMin/MaxDistanceInvariance scale them) */
    int32_t flags;                   /* ORBFE_MP_BAD (isBad()), ORBFE_MP_SKIP */
    int32_t observations;            /* Observations() */
    int32_t id;                      /* handle stored into mvpMapPoints */
    float track_depth;               /* mTrackDepth before this call: kept where the reference keeps it
                                        (a two-camera point whose left view fails; bFarPoints reads it) */
    uint8_t desc[32];                /* GetDescriptor() */
} orbfe_map_point_3d;                /* 80 bytes */

typedef struct orbfe_camera {
    float Rcw[9];                    /* Frame::mRcw, row-major */
    float tcw[3];                    /* Frame::mtcw */
    float Ow[3];                     /* Frame::mOw (camera centre in the world) */
    float fx, fy, cx, cy;            /* Pinhole mvParameters (Pinhole.cpp:43-49) */
    float log_scale_factor;          /* Frame::mfLogScaleFactor */
    float view_cos_limit;            /* 0.5 in SearchLocalPoints */
} orbfe_camera;

/* isInFrustum + PredictScale for n points: writes the tracking snapshot of each point to
 * track[i] (mbTrackInView -> ORBFE_MP_IN_VIEW, mTrackProjX/Y/XR, mTrackDepth, mTrackViewCos,
 * mnTrackScaleLevel; ORBFE_MP_BAD kept; desc / observations / id copied) and returns the number in
 * view (nToMatch). Arithmetic: float, no FMA contraction, Eigen's left-to-right sums, glibc logf. */
int orbfe_is_in_frustum(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                        orbfe_map_point* track);

/* Tracking::SearchLocalPoints' projection + matching in one device pass: isInFrustum over pts,
 * then (if any point is in view) SearchByProjection(F, points, th, bFarPoints, thFarPoints) with
 * ratio nnratio. mvp / mvp_obs as orbfe_search_by_projection_local. *n_to_match (may be NULL)
 * receives nToMatch. Returns nmatches. */
int orbfe_search_local_points(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts,
                              int32_t n, int32_t* mvp, const int32_t* mvp_obs, float th, int32_t bFarPoints,
                              float thFarPoints, float nnratio, int32_t* n_to_match);
/* Device-resident Tracking::SearchLocalPoints (see orbfe_search_by_projection_local_device):
 * d_pts, d_mvp, d_mvp_obs and F's arrays are device pointers; *n_to_match (host) as above. */
int orbfe_search_local_points_device(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* d_pts,
                                     int32_t n, int32_t* d_mvp, const int32_t* d_mvp_obs, float th,
                                     int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match,
                                     void* stream);

/* Camera models of GeometricCamera (CameraModels/Pinhole.cpp, KannalaBrandt8.cpp): params =
 * mvParameters, {fx, fy, cx, cy} for the pinhole model, {fx, fy, cx, cy, k0, k1, k2, k3} for
 * KannalaBrandt8, whose project() (KannalaBrandt8.cpp:67-82) runs on the device with bit-exact ports
 * of glibc's atan2f / cosf / sinf. */
#define ORBFE_CAM_PINHOLE 0
#define ORBFE_CAM_KANNALA_BRANDT8 1
typedef struct orbfe_camera_model {
    int32_t type;                    /* ORBFE_CAM_* */
    float params[8];
} orbfe_camera_model;                /* 36 bytes */

/* What Frame::isInFrustum reads of a frame besides orbfe_camera's pose: mpCamera, and for a
 * two-camera frame (orbfe_frame.two_cams: Nleft != -1) mpCamera2 and the rig (Frame.cc:1168-1242):
 * Rrl / trl = mTrl.rotationMatrix() / translation() (row-major), tlr = mTlr.translation(), Rwc = mRwc
 * (row-major). The right-view pose is derived in the reference's order: mR = Rrl * mRcw, mt = Rrl *
 * mtcw + trl, twc = mRwc * tlr + mOw (Eigen 3.3 fixed-size products). */
typedef struct orbfe_stereo_rig {
    orbfe_camera_model left;         /* Frame::mpCamera */
    orbfe_camera_model right;        /* Frame::mpCamera2 (two-camera frames) */
    float Rrl[9], trl[3];
    float tlr[3];
    float Rwc[9];
} orbfe_stereo_rig;

/* Frame::isInFrustum for any camera model (Frame.cc:512-586): a single-camera frame takes the
 * Nleft == -1 branch with rig->left as mpCamera (a monocular KannalaBrandt8 frame included); a
 * two-camera frame runs isInFrustumChecks for the left and the right camera (Frame.cc:1168-1242):
 * track[i] gets ORBFE_MP_IN_VIEW with proj_x / proj_y / scale_level / view_cos / depth (left) and
 * ORBFE_MP_IN_VIEW_R with proj_xr / proj_yr / scale_level_r / view_cos_r (right), scale levels -1
 * where a check fails (the reference resets mnTrackScaleLevel(R) to -1, :578-579). Returns nToMatch
 * (points with either view). cam supplies the pose (Rcw, tcw, Ow), mfLogScaleFactor and the cosine
 * limit; its pinhole fields are not read. A failed left check keeps depth = pts[i].track_depth, the
 * point's previous mTrackDepth, as the reference does (bFarPoints reads it). */
int orbfe_is_in_frustum_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                            const orbfe_map_point_3d* pts, int32_t n, orbfe_map_point* track);
/* Tracking::SearchLocalPoints (Tracking.cc:3407-3452) with the rig's camera models: the projection
 * above, then SearchByProjection(F, points, th, bFarPoints, thFarPoints) with its two-camera branches
 * when F->two_cams (ORBmatcher.cc:43-213). Host and device-resident forms as orbfe_search_local_points. */
int orbfe_search_local_points_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                  const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs,
                                  float th, int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match);
int orbfe_search_local_points_rig_device(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                         const orbfe_map_point_3d* d_pts, int32_t n, int32_t* d_mvp,
                                         const int32_t* d_mvp_obs, float th, int32_t bFarPoints, float thFarPoints,
                                         float nnratio, int32_t* n_to_match, void* stream);

/* Tracking::SearchLocalPoints as the drop-in shim calls it (shim/Tracking_orbfe.cc): the fused search
 * above (rig may be NULL: pinhole from cam, one camera) that also returns each point's isInFrustum
 * record in track[n] (as orbfe_is_in_frustum_rig writes it), from which the caller applies the
 * loop's side effects on its MapPoints (mbTrackInView(R), mTrackProj*, mnTrackScaleLevel(R),
 * mTrackViewCos(R), IncreaseVisible for points in view, Tracking.cc:3407-3425). */
int orbfe_search_local_points_track(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                    const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs,
                                    float th, int32_t bFarPoints, float thFarPoints, float nnratio,
                                    int32_t* n_to_match, orbfe_map_point* track);

/* ---------------------------------------------------------------------------------------------
 * Back-end matcher pieces (LocalMapping / LoopClosing threads)
 * ------------------------------------------------------------------------------------------- */
/* SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.cc:765-903, pinhole path): mp1 / mp2 =
 * GetMapPointMatches() handles with NULL and bad points as -1; out12[n1] = the handle of the KF2
 * point matched to each KF1 keypoint, or -1. Returns nmatches. */
int orbfe_search_by_bow_kf(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                           const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2, const uint8_t* desc2,
                           const int32_t* mp2, int32_t n2, const orbfe_feature_vector* fv2, int32_t* out12,
                           float nnratio, int32_t checkOri);

/* The same with keyframes that have a second camera (NLeft != -1, KannalaBrandt8 stereo): nleft1 /
 * nleft2 = NLeft (-1 = single camera). Their FeatureVector indices >= NLeft (the right keypoints,
 * descriptor rows [NLeft, n)) are skipped as the reference does (ORBmatcher.cc:800-802, 817-819:
 * idx >= mvKeysUn.size()); keys1 / keys2 hold n entries of which [0, NLeft) (mvKeysUn) are read. */
int orbfe_search_by_bow_kf2(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                            int32_t nleft1, const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2,
                            const uint8_t* desc2, const int32_t* mp2, int32_t n2, int32_t nleft2,
                            const orbfe_feature_vector* fv2, int32_t* out12, float nnratio, int32_t checkOri);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403) for n_points points at once: the
 * observed descriptors of point p are rows [offsets[p], offsets[p+1]) of desc (<= 2048 per point).
 * best[p] = the row (relative to offsets[p]) with the least median Hamming distance to the others
 * (median = sorted row [(N-1)/2], first on ties), -1 for a point without descriptors. */
int orbfe_distinctive_descriptors(const uint8_t* desc, const int32_t* offsets, int32_t n_points, int32_t* best);

/* SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse) (ORBmatcher.cc:907-1146).
 * Keyframes with a second camera (two_cams: keys = mvKeys ++ mvKeysRight, the reference's kp1 / kp2
 * selection :979-984, 1001-1006) take the NLeft branches: bStereo is false for them, KF1's epipole test
 * is skipped; their camera-pair epipolar test (KannalaBrandt8::TriangulateMatches: Eigen JacobiSVD
 * triangulation, :1036-1066) stays with the camera model on the host, so two-camera keyframes need
 * bCoarse (as LocalMapping passes for inertial maps); otherwise ORBFE_E_ARG. mp1 / mp2: GetMapPoint(idx) presence (any MapPoint,
 * bad or not, -> handle >= 0; NULL -> -1); keyframe uright = mvuRight (NULL = all monocular).
 * F12 (row-major) and ep are the values the reference derives once per call:
 * F12 = K1^-T [t12]x R12 K2^-1 (Pinhole::epipolarConstrain, Pinhole.cpp:107-129) and
 * ep = pKF2->mpCamera->project(T2w * Cw1). level_sigma2_2 = pKF2->mvLevelSigma2.
 * matches12[KF1->n] = the KF2 index matched to each KF1 keypoint or -1 (vMatchedPairs in
 * ascending idx1 order). Returns nmatches. */
int orbfe_search_for_triangulation(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                   const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                   const float* F12, const float* ep, const float* level_sigma2_2,
                                   int32_t bOnlyStereo, int32_t bCoarse, int32_t checkOri, int32_t* matches12);

/* The caller's epipolar test of one keypoint pair of SearchForTriangulation (bCoarse false):
 * pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, pKF1->mvLevelSigma2[kp1.octave],
 * pKF2->mvLevelSigma2[kp2.octave]) with the camera pair and relative pose the reference selects from
 * the keypoints' sides (ORBmatcher.cc:1036-1074). idx1 / idx2 index KF1->keys / KF2->keys (mvKeys ++
 * mvKeysRight for a two-camera keyframe). Nonzero = the pair passes. */
typedef int32_t (*orbfe_epipolar_fn)(void* ctx, int32_t idx1, int32_t idx2);

/* SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse = false) with the epipolar test
 * left to the caller: the form for keyframes with a second camera, whose KannalaBrandt8::epipolarConstrain
 * (TriangulateMatches, an Eigen JacobiSVD triangulation) runs on the host with the camera models. The
 * device lists, per KF1 keypoint of a shared vocabulary node, the KF2 candidates that pass every other
 * gate of the reference's loop (:1002-1033: no map point, bOnlyStereo, dist <= TH_LOW, the epipole
 * distance to ep unless KF1 has a second camera), in ascending (dist, reverse node order); the
 * reference keeps the last candidate of the smallest passing dist, which is the first of this order
 * that passes, so epipolar() is called only until then (never more often than the reference calls
 * it). Then the rotation-histogram filter with checkOri (:1114-1131). matches12 as
 * orbfe_search_for_triangulation. Returns nmatches, or ORBFE_E_CAPACITY when the candidate slots (the sum
 * over KF1 entries of their shared KF2 node's size) exceed 16 M: the caller then keeps its CPU body. */
int orbfe_search_for_triangulation_epi(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                       const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                       const float* ep, int32_t bOnlyStereo, int32_t checkOri,
                                       orbfe_epipolar_fn epipolar, void* ctx, int32_t* matches12);

/* A Sophus pose as the reference stores it: quaternion (x, y, z, w) + translation.
 * kind ORBFE_SE3: Sophus::SE3f, unit quaternion, p' = (p + w*uv + v x uv) + t with uv = 2 (v x p)
 *                 (sophus/so3.hpp:358-367, se3.hpp:321-324);
 * kind ORBFE_SIM3: Sophus::Sim3f, RxSO3 quaternion with scale |q|^2,
 *                 p' = (s*p + (w*uv + v x uv)) + t (rxso3.hpp:265-273, sim3.hpp:226-229). */
#define ORBFE_SE3 0
#define ORBFE_SIM3 1
typedef struct orbfe_pose {
    float q[4];
    float t[3];
    int32_t kind;
} orbfe_pose;                        /* 32 bytes */

/* What the back-end projections read of a keyframe besides orbfe_frame. */
typedef struct orbfe_kf_camera {
    orbfe_pose Tcw;                  /* world -> camera (GetPose(), or the SE3 made from Scw) */
    float Ow[3];                     /* camera centre for the distance / viewing checks */
    float fx, fy, cx, cy;
    float log_scale_factor;          /* mfLogScaleFactor */
} orbfe_kf_camera;

/* A last-frame point for the device-projected motion-model search (ORBmatcher.cc:1695-1712): the
 * MapPoint's world position, nLastOctave and the keypoint angle of LastFrame (mvKeys / mvKeysRight),
 * Observations(), the caller's handle, and valid = pMP && !LastFrame.mvbOutlier[i]. */
typedef struct orbfe_last_point {
    float pos[3];                    /* pMP->GetWorldPos() */
    int32_t octave;                  /* nLastOctave */
    float angle;                     /* LastFrame keypoint angle (rotation check) */
    int32_t observations;
    int32_t id;
    int32_t valid;
    uint8_t desc[32];                /* pMP->GetDescriptor() */
} orbfe_last_point;                  /* 64 bytes */

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono) with the projection on the device
 * (ORBmatcher.cc:1702-1718, 1794-1796): x3Dc = Tcw * x3Dw (Sophus SE3f action, Tcw = CurrentFrame.
 * GetPose()), invzc = 1.0 / x3Dc(2) (double, then float), uv = cam->project(x3Dc) (CurrentFrame.
 * mpCamera: pinhole or KannalaBrandt8), and for a two-camera cur the right-camera search around
 * cam->project(Trl * x3Dc) (Trl = GetRelativePoseTrl(); the reference projects it with mpCamera);
 * then exactly orbfe_search_by_projection_lastframe(_stereo). Trl is ignored (may be NULL) for a
 * single-camera cur. bForward / bBackward as the reference computes them from the poses. */
int orbfe_search_by_projection_lastframe_pose(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                              const orbfe_last_point* pts, int32_t n_pts, const orbfe_pose* Tcw,
                                              const orbfe_pose* Trl, const orbfe_camera_model* cam, float th,
                                              int32_t bForward, int32_t bBackward, int32_t checkOri);

/* The matching half of Fuse (ORBmatcher.cc:1148-1337 with sim3 = 0; :1339-1455, Fuse(pKF, Scw, ...)
 * with sim3 = 1; pinhole, bRight = false): for every point with id >= 0 not flagged BAD / SKIP (SKIP =
 * IsInKeyFrame(pKF), resp. already in pKF->GetMapPoints()), project, check and search the keyframe
 * exactly as the reference loop does, and report best_idx[i] (-1 unless bestDist <= TH_LOW) and
 * best_dist[i]. The map mutation that follows (Replace / AddObservation / vpReplacePoint) stays
 * with the caller, in point order: a point's search reads nothing an earlier commit changes, only
 * its isBad / IsInKeyFrame gate has to be re-read at commit time.
 * inv_level_sigma2 = pKF->mvInvLevelSigma2. Returns the number of points with best_idx >= 0. */
int orbfe_fuse(const orbfe_frame* KF, const orbfe_kf_camera* cam, const float* inv_level_sigma2,
               const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3, int32_t* best_idx,
               int32_t* best_dist);

/* Fuse with the keyframe's camera model and side (ORBmatcher.cc:1148-1298 with bRight, :1339-1455):
 * model = pCamera (mpCamera, or mpCamera2 with bRight; NULL = pinhole from cam), cam->Tcw / Ow = the
 * pose the reference uses (GetRightPose() / GetRightCameraCenter() with bRight). A keyframe with a second
 * camera (KF->two_cams) is searched on its left grid, or with bRight on its right grid (GetFeaturesInArea(
 * .., bRight), mvKeysRight) with best_idx reported as NLeft + the right index (:1283); its mvuRight is -1
 * (Frame.cc:1137), so the monocular reprojection gate applies. bRight needs sim3 = 0 and two_cams. */
int orbfe_fuse_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_camera_model* model,
                   const float* inv_level_sigma2, const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3,
                   int32_t bRight, int32_t* best_idx, int32_t* best_dist);

/* SearchByProjection(pKF, Scw, vpPoints, vpMatched, th, ratioHamming) (ORBmatcher.cc:427-523) and,
 * with point_kfs != NULL, the vpPointsKFs / vpMatchedKF overload (:525-646). cam->Tcw is the SE3
 * the reference builds from Scw; matched = vpMatched handles [KF->n] (in/out), matched_kf =
 * vpMatchedKF handles (in/out, with point_kfs). Points whose handle is already in matched, or
 * flagged BAD, are skipped (so are id < 0 entries, which the reference cannot hold); a keypoint taken by an earlier point is not a candidate for later
 * ones (sequential semantics preserved). Returns nmatches. */
int orbfe_search_by_projection_sim3(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_map_point_3d* pts,
                                    int32_t n, const int32_t* point_kfs, int32_t th, float ratioHamming,
                                    int32_t* matched, int32_t* matched_kf);
/* The same with the keyframe's camera model (model = pKF->mpCamera; NULL = the pinhole expression on
 * cam's intrinsics): the first overload projects with pKF->mpCamera->project (:465; KannalaBrandt8 on the
 * device with the glibc atan2f / cosf / sinf ports), the vpPointsKFs overload (point_kfs != NULL) with
 * fx * x * invz + cx for every camera (:571-576). A keyframe with a second camera (KF->two_cams) is
 * searched on its left grid with mvKeys (KeyFrame::GetFeaturesInArea(.., bRight = false),
 * KeyFrame.cc:707-751); orbfe_search_by_projection_sim3 refuses it without point_kfs. */
int orbfe_search_by_projection_sim3_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam,
                                        const orbfe_camera_model* model, const orbfe_map_point_3d* pts, int32_t n,
                                        const int32_t* point_kfs, int32_t th, float ratioHamming, int32_t* matched,
                                        int32_t* matched_kf);

/* SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (ORBmatcher.cc:1457-1674). pts1[KF1->n] /
 * pts2[KF2->n]: the keyframes' GetMapPointMatches() (id < 0 = NULL, flags BAD = isBad()).
 * cam1 = {T1w, pKF1 intrinsics (used for both projections), pKF1->mfLogScaleFactor};
 * cam2 = {T2w, log scale factor of pKF2}; S12 / S21 Sim3 poses. matches12 = vpMatches12 handles
 * (in/out); matched_idx2[i] = get<0>(vpMatches12[i]->GetIndexInKeyFrame(pKF2)) for the initial
 * matches (-1 otherwise). Keyframes with a second camera are searched on their left grids (mvKeys);
 * the reference projects every camera with the pinhole expression on pKF1's fx, fy, cx, cy
 * (:1514-1519,1594-1599), so no camera model is needed. Returns nFound. */
int orbfe_search_by_sim3(const orbfe_frame* KF1, const orbfe_frame* KF2, const orbfe_map_point_3d* pts1,
                         const orbfe_map_point_3d* pts2, const orbfe_kf_camera* cam1, const orbfe_kf_camera* cam2,
                         const orbfe_pose* S12, const orbfe_pose* S21, float th, int32_t* matches12,
                         const int32_t* matched_idx2);

/* ---------------------------------------------------------------------------------------------
 * Bag of words: DBoW2::TemplatedVocabulary<FORB> (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h) — the loader of ORB-SLAM3's binary vocabulary format and transform(),
 * called by Frame::ComputeBoW (Frame.cc) with levelsup = 4. The vocabulary tree lives in HBM.
 * ------------------------------------------------------------------------------------------- */
typedef struct orbfe_vocabulary orbfe_vocabulary;
#define ORBFE_TF_IDF 0               /* DBoW2::WeightingType */
#define ORBFE_TF 1
#define ORBFE_IDF 2
#define ORBFE_BINARY 3
#define ORBFE_L1_NORM 0              /* DBoW2::ScoringType */
#define ORBFE_L2_NORM 1
#define ORBFE_CHI_SQUARE 2
#define ORBFE_KL 3
#define ORBFE_BHATTACHARYYA 4
#define ORBFE_DOT_PRODUCT 5

/* TemplatedVocabulary::loadFromBinFile (TemplatedVocabulary.h:1478-1540) from an in-memory copy of
 * the file: int k, int L, int scoring, int weighting, then per node 1..: int parent, uchar isLeaf,
 * uchar desc[32], double weight. */
int orbfe_vocabulary_load_bin(const uint8_t* data, size_t size, orbfe_vocabulary** out);
/* The same tree from arrays (node 0 = root; parents[i] < i for i >= 1; children keep node order). */
int orbfe_vocabulary_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int32_t n_nodes,
                            const int32_t* parents, const uint8_t* is_leaf, const uint8_t* desc,
                            const double* weights, orbfe_vocabulary** out);
void orbfe_vocabulary_destroy(orbfe_vocabulary* voc);
int orbfe_vocabulary_info(const orbfe_vocabulary* voc, int32_t* k, int32_t* L, int32_t* n_nodes, int32_t* n_words);

/* transform(features, BowVector& v, FeatureVector& fv, levelsup) (TemplatedVocabulary.h:1139-1198,
 * :1218-1262) for n descriptors (n x 32 bytes). Outputs (capacity n each, fv_offsets n + 1):
 * BowVector as ascending word ids + weights (*bow_n entries), FeatureVector as ascending node ids
 * with offsets into fv_indices (*fv_n nodes). Returns 0. */
int orbfe_vocabulary_transform(const orbfe_vocabulary* voc, const uint8_t* desc, int32_t n, int32_t levelsup,
                               uint32_t* bow_word_ids, double* bow_weights, int32_t* bow_n,
                               uint32_t* fv_node_ids, int32_t* fv_offsets, uint32_t* fv_indices, int32_t* fv_n);

/* ---------------------------------------------------------------------------------------------
 * Stereo rectification: cv::remap(im, out, M1, M2, cv::INTER_LINEAR) with CV_32F
 * maps from initUndistortRectifyMap (System.cc:233-240, Settings.cc:506-509), BORDER_CONSTANT 0.
 * ------------------------------------------------------------------------------------------- */
/* Batched, device-resident: n images (device pointer tables in host memory), one map pair
 * (dw x dh floats each, row-major) shared by all; stream = hipStream_t or NULL. A source needs
 * sstride * (sh - 1) + sw readable bytes and a destination dstride * (dh - 1) + dw writable ones
 * (the last rows may end at the image width). The pointer tables are uploaded asynchronously into a
 * per-thread ring of 4 device tables keyed by the pointers, so calls that cycle through up to four
 * buffer sets upload nothing after the first call of each. */
int orbfe_remap_linear_batch(const uint8_t* const* d_src, int sw, int sh, int sstride, const float* d_mapx,
                             const float* d_mapy, int dw, int dh, uint8_t* const* d_dst, int dstride, int n,
                             void* stream);
/* Host convenience for one image. */
int orbfe_remap_linear(const uint8_t* src, int sw, int sh, int sstride, const float* mapx, const float* mapy, int dw,
                       int dh, uint8_t* dst, int dstride);

/* cv::undistortPoints(mat, mat, K, DistCoef, cv::Mat(), K) of Frame::UndistortKeyPoints
 * (Frame.cc:747-780) for n points (x, y float pairs): K4 = {fx, fy, cx, cy} (float, as mK),
 * dist = ndist (4, 5, 8 or 12) OpenCV coefficients k1 k2 p1 p2 [k3 [k4 k5 k6 [s1..s4]]]. OpenCV 4.2
 * semantics: double arithmetic, 5 fixed-point iterations. Returns n. (The reference skips the call
 * when k1 == 0; the caller keeps that test.) */
int orbfe_undistort_points(const float* pts, int n, const float* K4, const float* dist, int ndist, float* out);

/* Per calling thread: when enabled, every matcher call above records HIP events around its
 * kernels (after the input upload, before the result copy); orbfe_matcher_last_ms returns that
 * device time of the thread's last call in ms (-1 when not timed). For bench.py. */
int orbfe_matcher_set_timing(int enable);
float orbfe_matcher_last_ms(void);
/* Work counters of the single-camera SearchByProjection(local map) searches on this thread (host
 * and device-resident forms; off by default, one extra copy and synchronisation per call when on):
 * out[0] = window candidates enumerated from the level grids, out[1] = candidate pairs whose
 * Hamming distance was computed, both summed over the call's fixed-point passes, out[2] = passes
 * evaluated (the last one confirms convergence). ORBFE_E_ARG when the last call counted nothing. */
int orbfe_matcher_set_stats(int enable);
int orbfe_matcher_last_stats(long long* out);

/* Debug/inspection (tests only): copy an intermediate of image `image`, level `level` of the last
 * batch to host memory. what: 0 = per-cell FAST key counts (int32[n_cells]),
 * 1 = per-cell FAST key slots (uint32[n_cells * cell_cap], x_rel | y_rel << 12 | score << 24),
 * 2 = DistributeOctTree output (uint32[n], x | y << 12 | score << 24) followed by nothing,
 * 3 = per-level info int32[4] {n, n_lap, n_mono, n_raw},
 * 4 = octree phase timestamps uint64[64] of image 0 (only with ORBFE_OCT_STAMPS set at create).
 * Returns the element count. */
int orbfe_debug_copy(orbfe_extractor* h, int what, int image, int level, void* dst, int cap_bytes);

/* Test hook: sort n <= 4096 u64 values by their high 32 bits with the device's block-parallel
 * replica of libstdc++ std::sort (used by DistributeOctTree); result must equal std::sort. */
int orbfe_debug_block_sort(uint64_t* data, int n);

/* Library identification (build string). */
const char* orbfe_version(void);

/* Measurement helper (bench.py): streaming device-to-device copy of `bytes` (multiple of 16, both
 * pointers 16-byte aligned) with 16-byte loads / stores per lane, on `stream` (NULL = legacy
 * default). Its rate is the measured HBM copy ceiling the roofline is also quoted against. */
int orbfe_copy_stream(const void* d_src, void* d_dst, size_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBFE_H */
