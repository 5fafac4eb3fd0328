// ============================================================================================
// orb_oracle_remap.cpp — CPU ORACLE of cv::remap(src, dst, map1, map2, INTER_LINEAR) for 8UC1
// images with CV_32FC1 map pairs and BORDER_CONSTANT 0 (test infrastructure only; see
// orb_oracle.cpp's header). OpenCV 4.2 imgwarp.cpp restated from knowledge (parity unpinned):
// initInterTab1D / initInterTab2D (fixed point, INTER_REMAP_COEF_SCALE = 32768, the isum fix-up
// scanning k1, k2 in [ksize/2, ksize/2 + 2) over a zero-initialised static table, as OpenCV
// does), the RemapInvoker map conversion (X = saturate_cast<int>(mapx * 32)), remapBilinear with
// FixedPtCast<int, uchar, 15>. Call site: System.cc:239-240.
// ============================================================================================
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

const int INTER_BITS = 5, INTER_TAB_SIZE = 1 << INTER_BITS, INTER_REMAP_COEF_SCALE = 1 << 15;
short BilinearTab_i[INTER_TAB_SIZE * INTER_TAB_SIZE][2][2];   // zero-initialised static storage
bool tab_ready = false;

int cv_round(double v) { return (int)std::lrint(v); }
short sat_short(float v) {
    const int iv = cv_round(v);
    return (short)(iv < SHRT_MIN ? SHRT_MIN : (iv > SHRT_MAX ? SHRT_MAX : iv));
}
int sat_int(float v) {
    if (v >= 2147483520.f) return INT_MAX;
    if (v <= -2147483648.f) return INT_MIN;
    return cv_round(v);
}

void init_tab() {
    if (tab_ready) return;
    float _tab[8 * INTER_TAB_SIZE];
    const float scale = 1.f / INTER_TAB_SIZE;
    for (int i = 0; i < INTER_TAB_SIZE; i++) {   // initInterTab1D, INTER_LINEAR
        _tab[2 * i] = 1.f - i * scale;
        _tab[2 * i + 1] = i * scale;
    }
    const int ksize = 2;
    short* itab = BilinearTab_i[0][0];
    for (int i = 0; i < INTER_TAB_SIZE; i++)
        for (int j = 0; j < INTER_TAB_SIZE; j++, itab += ksize * ksize) {
            int isum = 0;
            for (int k1 = 0; k1 < ksize; k1++) {
                const float vy = _tab[i * ksize + k1];
                for (int k2 = 0; k2 < ksize; k2++) {
                    const float v = vy * _tab[j * ksize + k2];
                    isum += itab[k1 * ksize + k2] = sat_short(v * INTER_REMAP_COEF_SCALE);
                }
            }
            if (isum != INTER_REMAP_COEF_SCALE) {
                const int diff = isum - INTER_REMAP_COEF_SCALE;
                const int ksize2 = ksize / 2;
                int Mk1 = ksize2, Mk2 = ksize2, mk1 = ksize2, mk2 = ksize2;
                for (int k1 = ksize2; k1 < ksize2 + 2; k1++)
                    for (int k2 = ksize2; k2 < ksize2 + 2; k2++) {
                        if (itab[k1 * ksize + k2] < itab[mk1 * ksize + mk2]) mk1 = k1, mk2 = k2;
                        else if (itab[k1 * ksize + k2] > itab[Mk1 * ksize + Mk2]) Mk1 = k1, Mk2 = k2;
                    }
                if (diff < 0) itab[Mk1 * ksize + Mk2] = (short)(itab[Mk1 * ksize + Mk2] - diff);
                else itab[mk1 * ksize + mk2] = (short)(itab[mk1 * ksize + mk2] - diff);
            }
        }
    tab_ready = true;
}

}  // namespace

extern "C" {

int oro_remap_linear(const uint8_t* src, int sw, int sh, int sstride, const float* mapx, const float* mapy, int dw,
                     int dh, uint8_t* dst, int dstride) {
    init_tab();
    const int width1 = sw - 1 > 0 ? sw - 1 : 0, height1 = sh - 1 > 0 ? sh - 1 : 0;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            const int X = sat_int(mapx[(size_t)y * dw + x] * INTER_TAB_SIZE);
            const int Y = sat_int(mapy[(size_t)y * dw + x] * INTER_TAB_SIZE);
            const int sxi = X >> INTER_BITS, syi = Y >> INTER_BITS;
            const short sx = (short)(sxi < SHRT_MIN ? SHRT_MIN : (sxi > SHRT_MAX ? SHRT_MAX : sxi));
            const short sy = (short)(syi < SHRT_MIN ? SHRT_MIN : (syi > SHRT_MAX ? SHRT_MAX : syi));
            const int a = (Y & (INTER_TAB_SIZE - 1)) * INTER_TAB_SIZE + (X & (INTER_TAB_SIZE - 1));
            const short* w = BilinearTab_i[a][0];
            int v0, v1, v2, v3;
            if ((unsigned)sx < (unsigned)width1 && (unsigned)sy < (unsigned)height1) {
                const uint8_t* S = src + (size_t)sy * sstride + sx;
                v0 = S[0]; v1 = S[1]; v2 = S[sstride]; v3 = S[sstride + 1];
            } else if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
                dst[(size_t)y * dstride + x] = 0;
                continue;
            } else {
                v0 = sx >= 0 && sy >= 0 ? src[(size_t)sy * sstride + sx] : 0;
                v1 = sx + 1 < sw && sy >= 0 ? src[(size_t)sy * sstride + sx + 1] : 0;
                v2 = sx >= 0 && sy + 1 < sh ? src[(size_t)(sy + 1) * sstride + sx] : 0;
                v3 = sx + 1 < sw && sy + 1 < sh ? src[(size_t)(sy + 1) * sstride + sx + 1] : 0;
            }
            const int v = (v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3] + (1 << 14)) >> 15;
            dst[(size_t)y * dstride + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    return 0;
}

// cv::undistortPoints for CV_32FC2 points, K = P = {fx, fy, cx, cy} (float), identity R and tilt,
// default criteria (COUNT, 5): OpenCV 4.2 cvUndistortPointsInternal restated (Frame.cc:747-780).
int oro_undistort_points(const float* pts, int n, const float* K4, const float* dist, int ndist, float* out) {
    double k[14] = {0};
    for (int i = 0; i < ndist && i < 14; i++) k[i] = (double)dist[i];
    const double fx = K4[0], fy = K4[1], cx = K4[2], cy = K4[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double RR[3][3] = {{fx, 0, cx}, {0, fy, cy}, {0, 0, 1}};   // P * R with R = I (exact)
    const double T[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};        // invMatTilt
    for (int i = 0; i < n; i++) {
        double x = pts[2 * i], y = pts[2 * i + 1];
        const double u = x, v = y;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        // Matx33d * Vec3d: each component summed left to right
        const double v0 = T[0][0] * x + T[0][1] * y + T[0][2] * 1;
        const double v1 = T[1][0] * x + T[1][1] * y + T[1][2] * 1;
        const double v2 = T[2][0] * x + T[2][1] * y + T[2][2] * 1;
        const double invProj = v2 ? 1. / v2 : 1;
        double x0 = x = invProj * v0;
        double y0 = y = invProj * v1;
        for (int j = 0;; j++) {
            if (j >= 5) break;   // TermCriteria(COUNT, 5, 0.01)
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            if (icdist < 0) {
                x = (u - cx) * ifx;
                y = (v - cy) * ify;
                break;
            }
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        const double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        const double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        const double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        out[2 * i] = (float)(xx * ww);
        out[2 * i + 1] = (float)(yy * ww);
    }
    return n;
}

// the fixed-point table itself (tests: it must equal the closed form the HIP kernel uses)
void oro_remap_bilinear_tab(int16_t* out) {
    init_tab();
    memcpy(out, BilinearTab_i, sizeof(BilinearTab_i));
}

}  // extern "C"
