// image_decode.cpp — ImageTexture.create's image read (ImageTexture.java:22-85):
// `ImageIO.read` of a classpath resource, then `BufferedImage.getRGB` per pixel, so
// the texture's bytes are the decoded 8-bit R, G, B (and A) of the file.  The
// reference ships `textures/earthmap.jpg` (a baseline JFIF) and loads it for scenes
// 2 and 8 (Scene.java:117, :319); a host that builds its own scene may name any
// image.  This file decodes the formats javax.imageio reads by default that a
// texture can come in, with no library beyond zlib:
//
//   * JPEG (baseline, extended-sequential and progressive Huffman, 8-bit samples),
//     decoded the way the IJG decoder javax.imageio wraps does it by default:
//     the integer "islow" inverse DCT (the Loeffler-Ligtenberg-Moschytz factorisation
//     in 13-bit fixed point with two extra pass-1 bits), its wrap-around range
//     limiting, the fixed-point (16-bit) YCbCr -> RGB tables, and "fancy"
//     (triangle-filter) upsampling of 2x1 and 2x2 subsampled chroma with the edge
//     replication of its context rows.  Its output equals libjpeg-turbo's (Pillow's)
//     byte for byte (tests/test_image_decode.py); assets/earthmap.ppm is that decode of
//     the reference's earthmap.jpg and is the committed pin.
//   * PNG (8-bit truecolour, truecolour + alpha, palette of 1/2/4/8 bits with or
//     without tRNS; not interlaced), and binary PPM (P6, maxval 255).
//
// ImageTexture accepts 3 or 4 colour-model components only ("Unsupported image
// format" otherwise): a greyscale or grey + alpha image, a CMYK JPEG, 16-bit PNG
// samples and Adam7 interlacing are refused here with an error, not converted.
#include "rt/rt.h"
#include "rt/rt_scene.h"

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

struct Decoded {
    int w = 0, h = 0, comps = 0;   // comps: 3 (RGB) or 4 (RGBA)
    std::vector<uint8_t> px;      // w * h * comps, row 0 = top
};

[[noreturn]] void bad(const std::string& m) { throw std::runtime_error(m); }

// rt_upload_texture's limit (2^28 texels): larger images are refused before any pixel memory is taken
void check_size(long long w, long long h) {
    if (w <= 0 || h <= 0) bad("image has no pixels");
    if (w * h > (1LL << 28)) bad("image too large for a texture (more than 2^28 pixels)");
}

// ---------------------------------------------------------------------------------- JPEG

constexpr int kZigzag[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    // a corrupt run past 63 lands on coefficient 63 (the IJG decoder's padded table)
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huff {
    bool defined = false;
    uint8_t vals[256] = {};
    int mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
    void build(const uint8_t counts[16], const uint8_t* v, int n) {
        std::memcpy(vals, v, n);
        int code = 0, k = 0;
        for (int len = 1; len <= 16; len++) {
            valptr[len] = k;
            mincode[len] = code;
            code += counts[len - 1];
            k += counts[len - 1];
            maxcode[len] = counts[len - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        defined = true;
    }
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;                // blocks per line / column, MCU-padded
    int dw = 0, dh = 0;                // downsampled size (ceil(W * h / hmax), ...)
    std::vector<int16_t> coef;         // bw * bh blocks of 64, natural order
    int dc_tbl = 0, ac_tbl = 0, pred = 0;
    std::vector<uint8_t> plane;        // bw * 8 x bh * 8 samples after the IDCT
};

class Jpeg {
  public:
    Jpeg(const uint8_t* d, size_t n) : p_(d), end_(d + n) {}
    Decoded decode();

  private:
    const uint8_t* p_;
    const uint8_t* end_;
    uint16_t qt_[4][64] = {};
    Huff dc_[4], ac_[4];
    std::vector<Comp> comps_;
    int W_ = 0, H_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    bool progressive_ = false, jfif_ = false, adobe_ = false;
    int adobe_transform_ = -1;
    int restart_ = 0;
    // entropy-decoder state
    uint32_t bits_ = 0;
    int nbits_ = 0;
    bool hit_marker_ = false;
    int eobrun_ = 0;

    int u8() {
        if (p_ >= end_) bad("JPEG: unexpected end of data");
        return *p_++;
    }
    int u16() { int a = u8(); return (a << 8) | u8(); }
    // a marker segment's length word: the end of its payload, checked against the data
    const uint8_t* segment() {
        const int len = u16();
        if (len < 2 || len - 2 > end_ - p_) bad("JPEG: bad marker length");
        return p_ + (len - 2);
    }

    void fill() {
        while (nbits_ <= 24) {
            int b = 0;
            if (!hit_marker_ && p_ < end_) {
                b = *p_;
                if (b == 0xFF) {
                    int nx = p_ + 1 < end_ ? p_[1] : 0xD9;
                    if (nx == 0x00) {
                        p_ += 2;
                    } else {          // a marker: the data ends here, zeros follow (IJG behaviour)
                        hit_marker_ = true;
                        b = 0;
                    }
                } else {
                    p_++;
                }
            }
            bits_ |= (uint32_t)b << (24 - nbits_);
            nbits_ += 8;
        }
    }
    int bit() {
        if (nbits_ < 1) fill();
        int r = (int)(bits_ >> 31);
        bits_ <<= 1;
        nbits_--;
        return r;
    }
    int get(int n) {
        if (n == 0) return 0;
        if (nbits_ < n) fill();
        int r = (int)(bits_ >> (32 - n));
        bits_ <<= n;
        nbits_ -= n;
        return r;
    }
    static int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }
    int decode(const Huff& t) {
        if (!t.defined) bad("JPEG: scan uses an undefined Huffman table");
        int code = bit(), len = 1;
        while (code > t.maxcode[len]) {
            code = (code << 1) | bit();
            if (++len > 16) bad("JPEG: corrupt Huffman code");
        }
        return t.vals[t.valptr[len] + code - t.mincode[len]];
    }
    void reset_bits() {
        bits_ = 0;
        nbits_ = 0;
    }
    // at a restart interval's end: drop the partial byte, consume RSTn, reset predictors
    void restart() {
        reset_bits();
        hit_marker_ = false;
        while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] >= 0xD0 && p_[1] <= 0xD7)) {
            if (p_[0] == 0xFF && p_[1] != 0x00 && p_[1] != 0xFF) break;   // another marker: no RST
            p_++;
        }
        if (p_ + 1 < end_ && p_[0] == 0xFF && p_[1] >= 0xD0 && p_[1] <= 0xD7) p_ += 2;
        for (auto& c : comps_) c.pred = 0;
        eobrun_ = 0;
    }

    void read_sof(bool progressive) {
        const uint8_t* stop = segment();
        if (u8() != 8) bad("JPEG: only 8-bit samples are supported");
        H_ = u16();
        W_ = u16();
        int n = u8();
        if (W_ <= 0 || H_ <= 0) bad("JPEG: zero image size (DNL) is not supported");
        check_size(W_, H_);
        if (n != 1 && n != 3 && n != 4) bad("JPEG: unsupported component count");
        comps_.assign(n, Comp());
        for (auto& c : comps_) {
            c.id = u8();
            int hv = u8();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = u8() & 3;
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) bad("JPEG: bad sampling factors");
            hmax_ = std::max(hmax_, c.h);
            vmax_ = std::max(vmax_, c.v);
        }
        for (const auto& c : comps_)   // the IJG decoder takes integral ratios only (jdsample.c)
            if (hmax_ % c.h || vmax_ % c.v) bad("JPEG: fractional sampling factors are not supported");
        progressive_ = progressive;
        mcux_ = (W_ + 8 * hmax_ - 1) / (8 * hmax_);
        mcuy_ = (H_ + 8 * vmax_ - 1) / (8 * vmax_);
        for (auto& c : comps_) {
            c.bw = mcux_ * c.h;
            c.bh = mcuy_ * c.v;
            c.dw = (W_ * c.h + hmax_ - 1) / hmax_;
            c.dh = (H_ * c.v + vmax_ - 1) / vmax_;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        p_ = stop;
    }

    void read_dqt() {
        const uint8_t* stop = segment();
        while (p_ < stop) {
            int pq = u8(), t = pq & 15;
            if (t > 3) bad("JPEG: bad quantisation table id");
            for (int i = 0; i < 64; i++) qt_[t][kZigzag[i]] = (uint16_t)((pq >> 4) ? u16() : u8());
        }
    }

    void read_dht() {
        const uint8_t* stop = segment();
        while (p_ < stop) {
            int tc = u8(), cls = tc >> 4, id = tc & 15;
            if (id > 3 || cls > 1) bad("JPEG: bad Huffman table id");
            uint8_t counts[16];
            int total = 0;
            for (int i = 0; i < 16; i++) total += counts[i] = (uint8_t)u8();
            if (total > 256) bad("JPEG: bad Huffman table");
            uint8_t v[256];
            for (int i = 0; i < total; i++) v[i] = (uint8_t)u8();
            (cls ? ac_ : dc_)[id].build(counts, v, total);
        }
    }

    // a DC difference category above 11 (8-bit samples) is corrupt data
    int dc_diff(const Comp& c) {
        const int s = decode(dc_[c.dc_tbl]);
        if (s > 11) bad("JPEG: corrupt DC difference");
        return s ? extend(get(s), s) : 0;
    }
    // predictors wrap like the IJG decoder's int arithmetic on corrupt data, without overflow
    static int wrap_add(int a, int b) { return (int)(int16_t)(uint16_t)((unsigned)a + (unsigned)b); }

    void decode_block_seq(Comp& c, int16_t* blk) {
        int s;
        c.pred = wrap_add(c.pred, dc_diff(c));
        blk[0] = (int16_t)c.pred;
        for (int k = 1; k < 64; k++) {
            int rs = decode(ac_[c.ac_tbl]), r = rs >> 4;
            s = rs & 15;
            if (s) {
                k += r;
                blk[kZigzag[k]] = (int16_t)extend(get(s), s);
            } else {
                if (r != 15) break;
                k += 15;
            }
        }
    }

    void dc_first(Comp& c, int16_t* blk, int al) {
        c.pred = wrap_add(c.pred, dc_diff(c));
        blk[0] = (int16_t)(uint16_t)((unsigned)c.pred << al);
    }
    void dc_refine(int16_t* blk, int al) {
        if (bit()) blk[0] |= (int16_t)(1 << al);
    }
    void ac_first(Comp& c, int16_t* blk, int ss, int se, int al) {
        if (eobrun_ > 0) {
            eobrun_--;
            return;
        }
        for (int k = ss; k <= se; k++) {
            int rs = decode(ac_[c.ac_tbl]), r = rs >> 4, s = rs & 15;
            if (s) {
                k += r;
                blk[kZigzag[k]] = (int16_t)(uint16_t)((unsigned)extend(get(s), s) << al);
            } else {
                if (r != 15) {
                    eobrun_ = (1 << r) - 1;
                    if (r) eobrun_ += get(r);
                    break;
                }
                k += 15;
            }
        }
    }
    void refine_nonzero(int16_t* coef, int p1, int m1) {
        if (bit() && (*coef & p1) == 0) *coef = (int16_t)(*coef + (*coef >= 0 ? p1 : m1));
    }
    void ac_refine(Comp& c, int16_t* blk, int ss, int se, int al) {
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        int k = ss;
        if (eobrun_ == 0) {
            for (; k <= se; k++) {
                int rs = decode(ac_[c.ac_tbl]), r = rs >> 4, s = rs & 15;
                if (s) {
                    if (s != 1) bad("JPEG: corrupt refinement scan");
                    s = bit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun_ = 1 << r;
                    if (r) eobrun_ += get(r);
                    break;
                }
                do {
                    int16_t* coef = &blk[kZigzag[k]];
                    if (*coef != 0) {
                        refine_nonzero(coef, p1, m1);
                    } else if (--r < 0) {
                        break;
                    }
                    k++;
                } while (k <= se);
                if (s) blk[kZigzag[k]] = (int16_t)s;
            }
        }
        if (eobrun_ > 0) {
            for (; k <= se; k++) {
                int16_t* coef = &blk[kZigzag[k]];
                if (*coef != 0) refine_nonzero(coef, p1, m1);
            }
            eobrun_--;
        }
    }

    void read_sos() {
        int len = u16();
        (void)len;
        int ns = u8();
        if (ns < 1 || ns > 4) bad("JPEG: bad scan component count");
        std::vector<Comp*> sc;
        for (int i = 0; i < ns; i++) {
            int id = u8(), tt = u8();
            Comp* c = nullptr;
            for (auto& q : comps_)
                if (q.id == id) c = &q;
            if (!c) bad("JPEG: scan names an unknown component");
            c->dc_tbl = (tt >> 4) & 3;
            c->ac_tbl = tt & 3;
            sc.push_back(c);
        }
        int ss = u8(), se = u8(), a = u8(), ah = a >> 4, al = a & 15;
        if (ah > 13 || al > 13) bad("JPEG: bad successive-approximation bits");
        if (!progressive_) {
            ss = 0;
            se = 63;
        } else if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1)) {
            bad("JPEG: bad progression parameters");
        }
        reset_bits();
        hit_marker_ = false;
        eobrun_ = 0;
        for (auto* c : sc) c->pred = 0;

        auto block = [&](Comp& c, int bx, int by) {
            int16_t* blk = &c.coef[((size_t)by * c.bw + bx) * 64];
            if (!progressive_) decode_block_seq(c, blk);
            else if (ss == 0) (ah == 0 ? dc_first(c, blk, al) : dc_refine(blk, al));
            else if (ah == 0) ac_first(c, blk, ss, se, al);
            else ac_refine(c, blk, ss, se, al);
        };
        int todo = restart_;
        if (ns == 1) {   // non-interleaved: the component's own blocks, not MCU-padded
            Comp& c = *sc[0];
            int bw = (c.dw + 7) / 8, bh = (c.dh + 7) / 8;
            for (int by = 0; by < bh; by++)
                for (int bx = 0; bx < bw; bx++) {
                    if (restart_ && todo-- == 0) {
                        restart();
                        todo = restart_ - 1;
                    }
                    block(c, bx, by);
                }
        } else {
            for (int my = 0; my < mcuy_; my++)
                for (int mx = 0; mx < mcux_; mx++) {
                    if (restart_ && todo-- == 0) {
                        restart();
                        todo = restart_ - 1;
                    }
                    for (auto* c : sc)
                        for (int v = 0; v < c->v; v++)
                            for (int h = 0; h < c->h; h++) block(*c, mx * c->h + h, my * c->v + v);
                }
        }
        // leave the reader at the next marker (the bit reader never reads past one)
        while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] != 0x00 && !(p_[1] >= 0xD0 && p_[1] <= 0xD7))) p_++;
    }

    void idct_all();
    Decoded color_out();
};

// The islow inverse DCT: 13-bit constants, pass 1 on columns keeping 2 extra bits, pass 2 on
// rows, DESCALE = round half up by adding 2^(n-1) and shifting, then the decoder's
// post-IDCT range limit (index & 1023: -384..-129 -> 0, -128..127 -> x + 128, 128..511 -> 255,
// 512..895 -> 0, the rest wraps to x + 128).
constexpr int kConstBits = 13, kPass1Bits = 2;
constexpr int32_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373,
                  F1_175 = 9633, F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819,
                  F2_562 = 20995, F3_072 = 25172;

inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }

inline uint8_t idct_limit(int32_t x) {
    const int i = (int)((uint32_t)x & 1023u);
    if (i < 128) return (uint8_t)(i + 128);
    if (i < 512) return 255;
    if (i < 896) return 0;
    return (uint8_t)(i - 896);
}

// one 1-D 8-point pass over v[0..7] (stride s); writes the eight sums before descaling
inline void idct_1d(const int32_t* in, int s, int64_t out[8]) {
    int64_t z2 = in[2 * s], z3 = in[6 * s];
    int64_t z1 = (z2 + z3) * F0_541;
    int64_t tmp2 = z1 + z3 * -F1_847;
    int64_t tmp3 = z1 + z2 * F0_765;
    z2 = in[0];
    z3 = in[4 * s];
    int64_t tmp0 = (z2 + z3) * (1 << kConstBits);
    int64_t tmp1 = (z2 - z3) * (1 << kConstBits);
    int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = in[7 * s];
    tmp1 = in[5 * s];
    tmp2 = in[3 * s];
    tmp3 = in[1 * s];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    int64_t z5 = (z3 + z4) * F1_175;
    tmp0 *= F0_298;
    tmp1 *= F2_053;
    tmp2 *= F3_072;
    tmp3 *= F1_501;
    z1 *= -F0_899;
    z2 *= -F2_562;
    z3 *= -F1_961;
    z4 *= -F0_390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    out[0] = tmp10 + tmp3;
    out[7] = tmp10 - tmp3;
    out[1] = tmp11 + tmp2;
    out[6] = tmp11 - tmp2;
    out[2] = tmp12 + tmp1;
    out[5] = tmp12 - tmp1;
    out[3] = tmp13 + tmp0;
    out[4] = tmp13 - tmp0;
}

void Jpeg::idct_all() {
    for (auto& c : comps_) {
        const uint16_t* q = qt_[c.tq];
        const int pw = c.bw * 8;
        c.plane.assign((size_t)pw * c.bh * 8, 0);
        int32_t in[64], ws[64];
        int64_t o[8];
        for (int by = 0; by < c.bh; by++)
            for (int bx = 0; bx < c.bw; bx++) {
                const int16_t* blk = &c.coef[((size_t)by * c.bw + bx) * 64];
                for (int i = 0; i < 64; i++) in[i] = (int32_t)blk[i] * q[i];
                for (int x = 0; x < 8; x++) {          // pass 1: columns
                    bool ac0 = true;
                    for (int y = 1; y < 8; y++) ac0 = ac0 && in[y * 8 + x] == 0;
                    if (ac0) {
                        for (int y = 0; y < 8; y++) ws[y * 8 + x] = in[x] * (1 << kPass1Bits);
                        continue;
                    }
                    idct_1d(in + x, 8, o);
                    for (int y = 0; y < 8; y++) ws[y * 8 + x] = descale(o[y], kConstBits - kPass1Bits);
                }
                uint8_t* dst = &c.plane[(size_t)by * 8 * pw + (size_t)bx * 8];
                for (int y = 0; y < 8; y++) {          // pass 2: rows
                    idct_1d(ws + y * 8, 1, o);
                    for (int x = 0; x < 8; x++)
                        dst[(size_t)y * pw + x] = idct_limit(descale(o[x], kConstBits + kPass1Bits + 3));
                }
            }
    }
}

// Fancy upsampling of one component to full size (rows: the component's downsampled height,
// the row above the first / below the last replicated; columns likewise), IJG's h2v1 / h2v2
// triangle filters with their alternating rounding biases; other factors replicate.
std::vector<uint8_t> upsample(const Comp& c, int hmax, int vmax, int W, int H) {
    const int pw = c.bw * 8;
    const int fx = hmax / c.h, fy = vmax / c.v;
    std::vector<uint8_t> out((size_t)W * H);
    auto at = [&](int x, int y) { return (int)c.plane[(size_t)y * pw + x]; };
    if (fx == 1 && fy == 1) {
        for (int y = 0; y < H; y++) std::memcpy(&out[(size_t)y * W], &c.plane[(size_t)y * pw], W);
        return out;
    }
    const bool fancy = c.dw > 2;
    const int ow = c.dw * fx;   // the upsampler's output width before cropping to W
    std::vector<int> row(ow > W ? ow : W);
    if (fx == 2 && fy == 1 && fancy) {
        for (int y = 0; y < H; y++) {
            int n = c.dw;
            row[0] = at(0, y);
            row[1] = (at(0, y) * 3 + at(1, y) + 2) >> 2;
            for (int i = 1; i < n - 1; i++) {
                int v = at(i, y) * 3;
                row[2 * i] = (v + at(i - 1, y) + 1) >> 2;
                row[2 * i + 1] = (v + at(i + 1, y) + 2) >> 2;
            }
            row[2 * n - 2] = (at(n - 1, y) * 3 + at(n - 2, y) + 1) >> 2;
            row[2 * n - 1] = at(n - 1, y);
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)row[x];
        }
        return out;
    }
    if (fx == 2 && fy == 2 && fancy) {
        for (int y = 0; y < H; y++) {
            int iy = y >> 1;
            int ny = (y & 1) ? iy + 1 : iy - 1;   // the nearer neighbouring input row
            if (ny < 0) ny = 0;
            if (ny > c.dh - 1) ny = c.dh - 1;
            int n = c.dw;
            auto col = [&](int i) { return at(i, iy) * 3 + at(i, ny); };
            int thiscol = col(0), nextcol = col(1), lastcol;
            row[0] = (thiscol * 4 + 8) >> 4;
            row[1] = (thiscol * 3 + nextcol + 7) >> 4;
            lastcol = thiscol;
            thiscol = nextcol;
            for (int i = 1; i < n - 1; i++) {
                nextcol = col(i + 1);
                row[2 * i] = (thiscol * 3 + lastcol + 8) >> 4;
                row[2 * i + 1] = (thiscol * 3 + nextcol + 7) >> 4;
                lastcol = thiscol;
                thiscol = nextcol;
            }
            row[2 * n - 2] = (thiscol * 3 + lastcol + 8) >> 4;
            row[2 * n - 1] = (thiscol * 4 + 7) >> 4;
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)row[x];
        }
        return out;
    }
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)at(x / fx, y / fy);
    return out;
}

inline uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); }

Decoded Jpeg::color_out() {
    const int n = (int)comps_.size();
    if (n != 3)   // ImageTexture: 3 or 4 colour components; a 1-component JPEG is grey (1)
        bad(n == 1 ? "Unsupported image format (greyscale JPEG)" : "Unsupported image format (CMYK / YCCK JPEG)");
    std::vector<uint8_t> pl[3];
    for (int i = 0; i < 3; i++) pl[i] = upsample(comps_[i], hmax_, vmax_, W_, H_);
    // colour space as the IJG decoder guesses it: JFIF -> YCbCr; Adobe transform 0 -> RGB;
    // component ids 'R' 'G' 'B' -> RGB; otherwise YCbCr
    bool rgb = false;
    if (!jfif_ && adobe_) rgb = adobe_transform_ == 0;
    else if (!jfif_ && comps_[0].id == 'R' && comps_[1].id == 'G' && comps_[2].id == 'B') rgb = true;
    Decoded d;
    d.w = W_;
    d.h = H_;
    d.comps = 3;
    d.px.resize((size_t)W_ * H_ * 3);
    // jdcolor's 16-bit fixed point tables
    const int32_t half = 1 << 15;
    auto fix = [](double x) { return (int32_t)(x * 65536.0 + 0.5); };
    int cr_r[256], cb_b[256];
    int32_t cr_g[256], cb_g[256];
    for (int i = 0; i < 256; i++) {
        int32_t x = i - 128;
        cr_r[i] = (int)((fix(1.40200) * x + half) >> 16);
        cb_b[i] = (int)((fix(1.77200) * x + half) >> 16);
        cr_g[i] = -fix(0.71414) * x;
        cb_g[i] = -fix(0.34414) * x + half;
    }
    for (size_t i = 0; i < (size_t)W_ * H_; i++) {
        int y = pl[0][i], cb = pl[1][i], cr = pl[2][i];
        uint8_t* o = &d.px[i * 3];
        if (rgb) {
            o[0] = (uint8_t)y;
            o[1] = (uint8_t)cb;
            o[2] = (uint8_t)cr;
        } else {
            o[0] = clamp255(y + cr_r[cr]);
            o[1] = clamp255(y + (int)((cb_g[cb] + cr_g[cr]) >> 16));
            o[2] = clamp255(y + cb_b[cb]);
        }
    }
    return d;
}

Decoded Jpeg::decode() {
    if (u8() != 0xFF || u8() != 0xD8) bad("JPEG: no SOI marker");
    bool have_frame = false, any_scan = false;
    for (;;) {
        int m = u8();
        if (m != 0xFF) continue;   // garbage between markers (IJG skips it with a warning)
        m = u8();
        while (m == 0xFF) m = u8();
        if (m == 0xD9) break;   // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;
        switch (m) {
        case 0xC0:
        case 0xC1:
            read_sof(false);
            have_frame = true;
            break;
        case 0xC2:
            read_sof(true);
            have_frame = true;
            break;
        case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
        case 0xCE: case 0xCF:
            bad("JPEG: lossless / hierarchical / arithmetic coding is not supported");
        case 0xC4:
            read_dht();
            break;
        case 0xDB:
            read_dqt();
            break;
        case 0xDD: {
            const uint8_t* stop = segment();
            restart_ = u16();
            p_ = stop;
            break;
        }
        case 0xDA:
            if (!have_frame) bad("JPEG: scan before frame header");
            read_sos();
            any_scan = true;
            break;
        case 0xE0: {
            const uint8_t* stop = segment();
            if (stop - p_ >= 5 && std::memcmp(p_, "JFIF\0", 5) == 0) jfif_ = true;
            p_ = stop;
            break;
        }
        case 0xEE: {
            const uint8_t* stop = segment();
            if (stop - p_ >= 12 && std::memcmp(p_, "Adobe", 5) == 0) {
                adobe_ = true;
                adobe_transform_ = p_[11];
            }
            p_ = stop;
            break;
        }
        default: {   // APPn, COM, DNL, ...: skipped
            p_ = segment();
        }
        }
        if (p_ > end_) bad("JPEG: unexpected end of data");
        if (p_ >= end_) break;
    }
    if (!have_frame || !any_scan) bad("JPEG: no image data");
    idct_all();
    return color_out();
}

// ----------------------------------------------------------------------------------- PNG

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

Decoded decode_png(const uint8_t* d, size_t n) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, sig, 8)) bad("PNG: bad signature");
    size_t pos = 8;
    int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    while (pos + 12 <= n) {
        uint32_t len = be32(d + pos);
        const uint8_t* type = d + pos + 4;
        const uint8_t* body = d + pos + 8;
        if (pos + 12 + (size_t)len > n) bad("PNG: truncated chunk");
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) bad("PNG: bad IHDR");
            w = (int)be32(body);
            h = (int)be32(body + 4);
            depth = body[8];
            ctype = body[9];
            interlace = body[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(body, body + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    if (w <= 0 || h <= 0) bad("PNG: no IHDR");
    check_size(w, h);
    if (ctype == 0 || ctype == 4) bad("Unsupported image format (greyscale PNG)");
    if (depth == 16) bad("PNG: 16-bit samples are not supported");
    if (interlace) bad("PNG: interlaced images are not supported");
    int chans;
    if (ctype == 2 && depth == 8) chans = 3;
    else if (ctype == 6 && depth == 8) chans = 4;
    else if (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) chans = 1;
    else bad("PNG: unsupported colour type / bit depth");
    const size_t stride = ((size_t)w * chans * depth + 7) / 8;
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK || rawlen != raw.size())
        bad("PNG: bad image data");
    const int bpp = std::max(1, chans * depth / 8);
    std::vector<uint8_t> img(stride * h);
    for (int y = 0; y < h; y++) {
        int ft = raw[y * (stride + 1)];
        const uint8_t* src = &raw[y * (stride + 1) + 1];
        uint8_t* cur = &img[y * stride];
        const uint8_t* prev = y ? &img[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; i++) {
            int a = i >= (size_t)bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0,
                c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0, x = src[i], v;
            switch (ft) {
            case 0: v = x; break;
            case 1: v = x + a; break;
            case 2: v = x + b; break;
            case 3: v = x + ((a + b) >> 1); break;
            case 4: {
                int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                v = x + ((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
                break;
            }
            default: bad("PNG: bad filter type");
            }
            cur[i] = (uint8_t)v;
        }
    }
    Decoded out;
    out.w = w;
    out.h = h;
    if (chans != 1) {
        out.comps = chans;
        out.px = std::move(img);
        return out;
    }
    // palette: IndexColorModel, 4 components when tRNS gives it alpha, else 3
    const int ncol = (int)plte.size() / 3;
    if (ncol == 0) bad("PNG: palette image without PLTE");
    out.comps = trns.empty() ? 3 : 4;
    out.px.resize((size_t)w * h * out.comps);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint8_t* row = &img[y * stride];
            int idx = depth == 8 ? row[x] : (row[(x * depth) / 8] >> (8 - depth - (x * depth) % 8)) & ((1 << depth) - 1);
            uint8_t* o = &out.px[((size_t)y * w + x) * out.comps];
            if (idx >= ncol) idx = 0;
            o[0] = plte[idx * 3];
            o[1] = plte[idx * 3 + 1];
            o[2] = plte[idx * 3 + 2];
            if (out.comps == 4) o[3] = idx < (int)trns.size() ? trns[idx] : 255;
        }
    return out;
}

// ----------------------------------------------------------------------------------- PPM

Decoded decode_ppm(const uint8_t* d, size_t n) {
    size_t pos = 2;
    auto num = [&]() {
        for (;;) {
            while (pos < n && std::isspace(d[pos])) pos++;
            if (pos < n && d[pos] == '#') {
                while (pos < n && d[pos] != '\n') pos++;
                continue;
            }
            break;
        }
        long v = 0;
        if (pos >= n || !std::isdigit(d[pos])) bad("PPM: bad header");
        while (pos < n && std::isdigit(d[pos])) {
            v = v * 10 + (d[pos++] - '0');
            if (v > (1L << 30)) bad("PPM: bad header");
        }
        return v;
    };
    long w = num(), h = num(), maxv = num();
    pos++;
    if (maxv != 255 || w <= 0 || h <= 0) bad("PPM: only 8-bit P6 is supported");
    check_size(w, h);
    if (pos + (size_t)w * h * 3 > n) bad("PPM: truncated image");
    Decoded out;
    out.w = (int)w;
    out.h = (int)h;
    out.comps = 3;
    out.px.assign(d + pos, d + pos + (size_t)w * h * 3);
    return out;
}

Decoded decode_file(const char* path) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) bad(std::string("Failed to load image: ") + path);
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, fp)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    std::fclose(fp);
    if (buf.size() >= 2 && buf[0] == 0xFF && buf[1] == 0xD8) return Jpeg(buf.data(), buf.size()).decode();
    if (buf.size() >= 8 && buf[0] == 137 && buf[1] == 'P' && buf[2] == 'N' && buf[3] == 'G')
        return decode_png(buf.data(), buf.size());
    if (buf.size() >= 2 && buf[0] == 'P' && buf[1] == '6') return decode_ppm(buf.data(), buf.size());
    bad(std::string("Failed to load image: ") + path + " (not a JPEG, PNG or P6 PPM file)");
}

thread_local std::string g_err;

}  // namespace

// the scene builder's ImageTexture.create reads through here (scene_builder.cpp image_create)
namespace rts_detail {
int decode_image_file(const char* path, int* w, int* h, int* comps, std::vector<uint8_t>* px) {
    Decoded d = decode_file(path);
    *w = d.w;
    *h = d.h;
    *comps = d.comps;
    *px = std::move(d.px);
    return 0;
}
}  // namespace rts_detail

extern "C" int rts_decode_image(const char* path, int* width, int* height, int* channels, uint8_t* pixels,
                                size_t capacity) {
    if (!path || !width || !height || !channels) {
        g_err = "NULL argument";
        return RT_ERR_INVALID_ARG;
    }
    try {
        Decoded d = decode_file(path);
        *width = d.w;
        *height = d.h;
        *channels = d.comps;
        if (pixels) {
            if (capacity < d.px.size()) {
                g_err = "pixel buffer too small";
                return RT_ERR_INVALID_ARG;
            }
            std::memcpy(pixels, d.px.data(), d.px.size());
        }
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_ERR_INVALID_ARG;
    }
}

extern "C" const char* rts_decode_last_error(void) { return g_err.c_str(); }
