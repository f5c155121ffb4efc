// Texture image decoding: what Texture2D(path) gets from stb_image v2.30
// (external/OpenGL/textureClass.cpp:55-68: stbi_set_flip_vertically_on_load
// (true); stbi_load(path, &w, &h, &n, 0)), restated behind rt2_image_load.
// Results are byte-identical to the reference's stb_image on every case of
// tests/golden/ (the reference's own textures and synthetic PNG/JPEG files):
//   PNG  — bit depths 1/2/4/8/16, colour types 0/2/3/4/6, tRNS (palette alpha
//          or colour key), Adam7 interlace, all five row filters; low-depth
//          grey scaled to 0..255, 16-bit reduced by >> 8, palette expanded to
//          RGB(A); channel count as stb reports it.
//   JPEG — baseline and extended sequential Huffman, 8-bit, 1 or 3
//          components, any sampling factors (stb's upsampling filters),
//          restart intervals, the libjpeg "islow" integer IDCT with stb's
//          scaling and rounding, stb's fixed-point YCbCr -> RGB.  Progressive
//          and arithmetic-coded JPEGs are rejected with an error (none of the
//          reference's textures uses them).
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

#include "host_internal.h"

namespace rt2h {
namespace {

struct Fail : std::runtime_error {
    using std::runtime_error::runtime_error;
};
[[noreturn]] void fail(const std::string& m) { throw Fail(m); }

// int arithmetic that wraps (as stb's C int arithmetic does on this
// compiler) instead of overflowing: only corrupt streams get near the limits
inline int wadd(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }
inline int wsub(int a, int b) { return (int)((uint32_t)a - (uint32_t)b); }
inline int wmul(int a, int b) { return (int)((uint32_t)a * (uint32_t)b); }

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

constexpr int kMaxDim = 1 << 24;                    // STBI_MAX_DIMENSIONS
constexpr unsigned long long kMaxBytes = 1ull << 31;  // decoded-size limit (stb's int-sized allocations)

// ----------------------------------------------------------------------------
// PNG
// ----------------------------------------------------------------------------

std::vector<uint8_t> zlib_inflate(const std::vector<uint8_t>& in, size_t guess) {
    // the guess comes from the (untrusted) header: start small, grow with the data
    std::vector<uint8_t> out(std::min<size_t>(std::max<size_t>(guess, 1024), 1u << 24));
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) fail("zlib init");
    zs.next_in = const_cast<Bytef*>(in.data());
    zs.avail_in = (uInt)in.size();
    size_t have = 0;
    for (;;) {
        zs.next_out = out.data() + have;
        zs.avail_out = (uInt)(out.size() - have);
        const int rc = inflate(&zs, Z_NO_FLUSH);
        have = out.size() - zs.avail_out;
        if (rc == Z_STREAM_END) break;
        if (rc != Z_OK && rc != Z_BUF_ERROR) {
            inflateEnd(&zs);
            fail("Corrupt PNG (zlib stream)");
        }
        if (zs.avail_out == 0) {
            if (out.size() >= kMaxBytes) {
                inflateEnd(&zs);
                fail("Corrupt PNG (image data too large)");
            }
            out.resize(out.size() * 2);
        } else if (zs.avail_in == 0) {
            inflateEnd(&zs);
            fail("Corrupt PNG (truncated zlib stream)");
        }
    }
    inflateEnd(&zs);
    out.resize(have);
    return out;
}

inline int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

// Un-filters `rows` scanlines of `rowbytes` bytes (filter byte first) in place
// into `out`; `bpp` = bytes per complete pixel (>= 1).
void png_unfilter(const uint8_t* src, size_t src_len, int rows, size_t rowbytes, int bpp, std::vector<uint8_t>& out) {
    if (src_len < (rowbytes + 1) * (size_t)rows) fail("Corrupt PNG (not enough pixels)");
    out.assign(rowbytes * rows, 0);
    for (int y = 0; y < rows; y++) {
        const uint8_t f = src[y * (rowbytes + 1)];
        const uint8_t* in = src + y * (rowbytes + 1) + 1;
        uint8_t* cur = out.data() + y * rowbytes;
        const uint8_t* prev = y ? cur - rowbytes : nullptr;
        if (f > 4) fail("Corrupt PNG (invalid filter)");
        for (size_t i = 0; i < rowbytes; i++) {
            const int a = i >= (size_t)bpp ? cur[i - bpp] : 0;
            const int b = prev ? prev[i] : 0;
            const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
            int v = in[i];
            switch (f) {
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: break;
            }
            cur[i] = (uint8_t)v;
        }
    }
}

Image decode_png(const std::vector<uint8_t>& d) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) fail("not a PNG");
    size_t pos = 8;
    uint32_t w = 0, h = 0;
    int depth = 0, color = -1, interlace = 0;
    int img_n = 0, pal_n = 0;  // pal_n: 0 (no palette), 3 or 4
    uint8_t palette[256][4] = {};
    int pal_len = 0;
    bool has_trans = false;
    uint16_t tc16[3] = {0, 0, 0};
    uint8_t tc8[3] = {0, 0, 0};
    std::vector<uint8_t> idat;
    bool first = true, ended = false;
    static const uint8_t depth_scale[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};
    while (!ended) {
        if (pos + 8 > d.size()) fail("Corrupt PNG (truncated)");
        const uint32_t len = be32(&d[pos]);
        const uint32_t type = be32(&d[pos + 4]);
        const uint8_t* c = &d[pos + 8];
        if (pos + 12 + (size_t)len > d.size()) fail("Corrupt PNG (chunk past end)");
        auto is = [&](const char* t) { return type == be32((const uint8_t*)t); };
        if (first && !is("IHDR")) fail("Corrupt PNG (first not IHDR)");
        if (is("IHDR")) {
            if (!first) fail("Corrupt PNG (multiple IHDR)");
            first = false;
            if (len != 13) fail("Corrupt PNG (bad IHDR len)");
            w = be32(c);
            h = be32(c + 4);
            if (w > (uint32_t)kMaxDim || h > (uint32_t)kMaxDim) fail("Very large image (corrupt?)");
            depth = c[8];
            color = c[9];
            if (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16) fail("PNG: 1/2/4/8/16-bit only");
            if (color > 6) fail("Corrupt PNG (bad ctype)");
            if (color == 3 && depth == 16) fail("Corrupt PNG (bad ctype)");
            if (color == 3) {
                pal_n = 3;
            } else if (color & 1) {
                fail("Corrupt PNG (bad ctype)");
            }
            if (c[10]) fail("Corrupt PNG (bad comp method)");
            if (c[11]) fail("Corrupt PNG (bad filter method)");
            interlace = c[12];
            if (interlace > 1) fail("Corrupt PNG (bad interlace method)");
            if (!w || !h) fail("Corrupt PNG (0-pixel image)");
            img_n = pal_n ? 1 : ((color & 2) ? 3 : 1) + ((color & 4) ? 1 : 0);
        } else if (is("PLTE")) {
            if (len > 256 * 3 || len % 3) fail("Corrupt PNG (invalid PLTE)");
            pal_len = (int)(len / 3);
            for (int i = 0; i < pal_len; i++) {
                palette[i][0] = c[3 * i];
                palette[i][1] = c[3 * i + 1];
                palette[i][2] = c[3 * i + 2];
                palette[i][3] = 255;
            }
        } else if (is("tRNS")) {
            if (!idat.empty()) fail("Corrupt PNG (tRNS after IDAT)");
            if (pal_n) {
                if (pal_len == 0) fail("Corrupt PNG (tRNS before PLTE)");
                if ((int)len > pal_len) fail("Corrupt PNG (bad tRNS len)");
                pal_n = 4;
                for (uint32_t i = 0; i < len; i++) palette[i][3] = c[i];
            } else {
                if (!(img_n & 1)) fail("Corrupt PNG (tRNS with alpha)");
                if (len != (uint32_t)img_n * 2) fail("Corrupt PNG (bad tRNS len)");
                has_trans = true;
                for (int k = 0; k < img_n; k++) {
                    tc16[k] = be16(c + 2 * k);
                    if (depth < 16) tc8[k] = (uint8_t)((tc16[k] & 255) * depth_scale[depth]);
                }
            }
        } else if (is("IDAT")) {
            if (pal_n && !pal_len) fail("Corrupt PNG (no PLTE)");
            idat.insert(idat.end(), c, c + len);
        } else if (is("IEND")) {
            ended = true;
        } else if ((d[pos + 4] & 32) == 0) {
            fail("PNG: unknown critical chunk");
        }
        pos += 12 + (size_t)len;
    }
    if (idat.empty()) fail("Corrupt PNG (no IDAT)");
    if ((unsigned long long)w * h * (img_n + 1) * (depth == 16 ? 2 : 1) > kMaxBytes) fail("PNG too large");
    const std::vector<uint8_t> raw = zlib_inflate(idat, ((size_t)w * depth * img_n + 15) / 8 * h + h);

    // samples at the file's depth: 8-bit (scaled low depths) or 16-bit
    const int out_n = has_trans ? img_n + 1 : img_n;
    const bool wide = depth == 16;
    std::vector<uint16_t> px((size_t)w * h * out_n, 0);
    const int filt_bpp = std::max(1, img_n * depth / 8);
    static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
    size_t off = 0;
    const int passes = interlace ? 7 : 1;
    for (int ps = 0; ps < passes; ps++) {
        const int x0 = interlace ? xo[ps] : 0, y0 = interlace ? yo[ps] : 0;
        const int dx = interlace ? xs[ps] : 1, dy = interlace ? ys[ps] : 1;
        const int pw = (int)(((int64_t)w - x0 + dx - 1) / dx), ph = (int)(((int64_t)h - y0 + dy - 1) / dy);
        if (pw <= 0 || ph <= 0) continue;
        const size_t rowbytes = ((size_t)img_n * pw * depth + 7) / 8;
        std::vector<uint8_t> un;
        if (off > raw.size()) fail("Corrupt PNG (not enough pixels)");
        png_unfilter(raw.data() + off, raw.size() - off, ph, rowbytes, filt_bpp, un);
        off += (rowbytes + 1) * ph;
        for (int y = 0; y < ph; y++) {
            const uint8_t* row = un.data() + y * rowbytes;
            for (int x = 0; x < pw; x++) {
                uint16_t* o = &px[(((size_t)(y0 + y * dy)) * w + (x0 + x * dx)) * out_n];
                for (int k = 0; k < img_n; k++) {
                    const size_t si = (size_t)x * img_n + k;
                    uint16_t v;
                    if (depth == 16) {
                        v = be16(row + 2 * si);
                    } else if (depth == 8) {
                        v = row[si];
                    } else {
                        const size_t bit = si * depth;
                        v = (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
                        if (color == 0) v = (uint16_t)(v * depth_scale[depth]);
                    }
                    o[k] = v;
                }
                if (has_trans) o[img_n] = wide ? 0xffff : 0xff;
            }
        }
    }
    if (has_trans) {  // colour key -> alpha 0 (compared at 8-bit-scaled or 16-bit values)
        for (size_t i = 0; i < (size_t)w * h; i++) {
            uint16_t* o = &px[i * out_n];
            bool eq = true;
            for (int k = 0; k < img_n; k++) eq = eq && o[k] == (wide ? tc16[k] : tc8[k]);
            if (eq) o[img_n] = 0;
        }
    }
    Image im;
    im.w = (int)w;
    im.h = (int)h;
    if (pal_n) {
        im.n = pal_n;
        im.px.resize((size_t)w * h * pal_n);
        for (size_t i = 0; i < (size_t)w * h; i++) {
            const int idx = px[i];
            for (int k = 0; k < pal_n; k++) im.px[i * pal_n + k] = palette[idx][k];  // out-of-range index reads 0s like stb's zeroed table
        }
    } else {
        im.n = out_n;
        im.px.resize((size_t)w * h * out_n);
        for (size_t i = 0; i < im.px.size(); i++) im.px[i] = wide ? (uint8_t)(px[i] >> 8) : (uint8_t)px[i];
    }
    return im;
}

// ----------------------------------------------------------------------------
// JPEG (ITU T.81 sequential Huffman)
// ----------------------------------------------------------------------------

struct Huffman {
    // canonical code tables: for code length L (1..16), codes in
    // [mincode[L], maxcode[L]] map to vals[valptr[L] + code - mincode[L]]
    int mincode[17], maxcode[18], valptr[17];
    uint8_t vals[256];
    bool defined = false;
};

// zig-zag position -> natural index, padded so a corrupt run past 63 lands on 63
const uint8_t kDezigzag[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct JComp {
    int id, h, v, tq;
    int hd = 0, ha = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0;  // extent and padded plane size
    int dc_pred = 0;
    std::vector<uint8_t> plane;
};

class JpegDecoder {
public:
    explicit JpegDecoder(const std::vector<uint8_t>& d) : d_(d) {}
    Image decode();

private:
    const std::vector<uint8_t>& d_;
    size_t pos_ = 0;
    uint16_t dq_[4][64] = {};
    Huffman hdc_[4], hac_[4];
    std::vector<JComp> comp_;
    int w_ = 0, h_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    int restart_ = 0;
    bool jfif_ = false;
    int app14_ = -1;  // Adobe colour transform, -1 = no APP14
    // entropy-coded segment reader
    uint32_t bitbuf_ = 0;
    int bits_ = 0;
    int marker_ = -1;  // marker met inside the entropy-coded data, -1 = none
    bool eob_ = false;

    uint8_t byte() {
        if (pos_ >= d_.size()) fail("Corrupt JPEG (truncated)");
        return d_[pos_++];
    }
    uint16_t word() {
        const uint16_t a = byte();
        return (uint16_t)(a << 8 | byte());
    }
    int next_marker();
    void read_dqt(int len);
    void read_dht(int len);
    void read_sof(int len);
    void read_sos(int len, std::vector<int>& scomp);
    void decode_scan(const std::vector<int>& scomp);
    void reset_bits() {
        bitbuf_ = 0;
        bits_ = 0;
        marker_ = -1;
        eob_ = false;
    }
    void fill() {  // top-aligned bit buffer; 0xFF00 stuffing; zeros after a marker
        while (bits_ <= 24) {
            uint32_t b = 0;
            if (marker_ < 0 && pos_ < d_.size()) {
                b = d_[pos_++];
                if (b == 0xFF) {
                    uint32_t c = pos_ < d_.size() ? d_[pos_] : 0xD9;
                    while (c == 0xFF && pos_ + 1 < d_.size()) c = d_[++pos_];  // fill bytes
                    pos_++;
                    if (c != 0) {
                        marker_ = (int)c;
                        b = 0;
                    }
                }
            }
            bitbuf_ |= b << (24 - bits_);
            bits_ += 8;
        }
    }
    int getbits(int n) {
        if (n == 0) return 0;
        if (bits_ < n) fill();
        const int v = (int)(bitbuf_ >> (32 - n));
        bitbuf_ <<= n;
        bits_ -= n;
        return v;
    }
    int huff(const Huffman& t) {
        if (bits_ < 16) fill();
        int code = 0;
        for (int L = 1; L <= 16; L++) {
            code = (code << 1) | (int)(bitbuf_ >> 31);
            bitbuf_ <<= 1;
            bits_ -= 1;
            if (t.maxcode[L] >= 0 && code <= t.maxcode[L] && code >= t.mincode[L])
                return t.vals[t.valptr[L] + code - t.mincode[L]];
        }
        fail("Corrupt JPEG (bad huffman code)");
    }
    static int extend(int v, int n) { return v < (1 << (n - 1)) ? v - (1 << n) + 1 : v; }
    void block(JComp& c, int16_t out[64]);
};

int JpegDecoder::next_marker() {
    // skip to the next 0xFF xx (xx != 0, != 0xFF)
    for (;;) {
        uint8_t b = byte();
        if (b != 0xFF) continue;
        do b = byte();
        while (b == 0xFF);
        if (b != 0) return b;
    }
}

void JpegDecoder::read_dqt(int len) {
    int left = len - 2;
    while (left > 0) {
        const int pq_tq = byte();
        const int p = pq_tq >> 4, t = pq_tq & 15;
        if (p != 0 && p != 1) fail("Corrupt JPEG (bad DQT type)");
        if (t > 3) fail("Corrupt JPEG (bad DQT table)");
        for (int i = 0; i < 64; i++) dq_[t][kDezigzag[i]] = p ? word() : byte();
        left -= p ? 129 : 65;
    }
    if (left != 0) fail("Corrupt JPEG (bad DQT length)");
}

void JpegDecoder::read_dht(int len) {
    int left = len - 2;
    while (left > 0) {
        const int tc_th = byte();
        const int tc = tc_th >> 4, th = tc_th & 15;
        if (tc > 1 || th > 3) fail("Corrupt JPEG (bad DHT header)");
        Huffman& t = tc ? hac_[th] : hdc_[th];
        int counts[17] = {0}, n = 0;
        for (int L = 1; L <= 16; L++) n += counts[L] = byte();
        if (n > 256) fail("Corrupt JPEG (bad code lengths)");
        for (int i = 0; i < n; i++) t.vals[i] = byte();
        int code = 0, k = 0;
        for (int L = 1; L <= 16; L++) {
            t.valptr[L] = k;
            t.mincode[L] = code;
            code += counts[L];
            k += counts[L];
            t.maxcode[L] = counts[L] ? code - 1 : -1;
            if (code > (1 << L)) fail("Corrupt JPEG (bad code lengths)");
            code <<= 1;
        }
        t.maxcode[17] = 0x7fffffff;
        t.defined = true;
        left -= 17 + n;
    }
    if (left != 0) fail("Corrupt JPEG (bad DHT length)");
}

void JpegDecoder::read_sof(int len) {
    const int p = byte();
    if (p != 8) fail("JPEG format not supported: 8-bit only");
    h_ = word();
    w_ = word();
    if (h_ == 0) fail("JPEG format not supported: delayed height");
    if (w_ == 0) fail("Corrupt JPEG (0 width)");
    if (h_ > kMaxDim || w_ > kMaxDim) fail("Very large image (corrupt?)");
    if ((unsigned long long)w_ * h_ * 4 > kMaxBytes) fail("JPEG too large");
    const int nc = byte();
    if (nc != 1 && nc != 3) fail("JPEG: only 1 or 3 components are supported");
    if (len != 8 + 3 * nc) fail("Corrupt JPEG (bad SOF len)");
    comp_.assign(nc, JComp());
    for (int i = 0; i < nc; i++) {
        comp_[i].id = byte();
        const int hv = byte();
        comp_[i].h = hv >> 4;
        comp_[i].v = hv & 15;
        comp_[i].tq = byte();
        if (!comp_[i].h || comp_[i].h > 4) fail("Corrupt JPEG (bad H)");
        if (!comp_[i].v || comp_[i].v > 4) fail("Corrupt JPEG (bad V)");
        if (comp_[i].tq > 3) fail("Corrupt JPEG (bad TQ)");
    }
    hmax_ = vmax_ = 1;
    for (auto& c : comp_) {
        hmax_ = std::max(hmax_, c.h);
        vmax_ = std::max(vmax_, c.v);
    }
    for (auto& c : comp_) {
        if (hmax_ % c.h) fail("Corrupt JPEG (bad H)");
        if (vmax_ % c.v) fail("Corrupt JPEG (bad V)");
    }
    mcux_ = (w_ + hmax_ * 8 - 1) / (hmax_ * 8);
    mcuy_ = (h_ + vmax_ * 8 - 1) / (vmax_ * 8);
    for (auto& c : comp_) {
        c.x = (w_ * c.h + hmax_ - 1) / hmax_;
        c.y = (h_ * c.v + vmax_ - 1) / vmax_;
        c.w2 = mcux_ * c.h * 8;
        c.h2 = mcuy_ * c.v * 8;
        c.plane.assign((size_t)c.w2 * c.h2, 0);
    }
}

void JpegDecoder::read_sos(int len, std::vector<int>& scomp) {
    const int ns = byte();
    if (ns < 1 || ns > 4 || ns > (int)comp_.size()) fail("Corrupt JPEG (bad SOS component count)");
    if (len != 6 + 2 * ns) fail("Corrupt JPEG (bad SOS len)");
    scomp.clear();
    for (int i = 0; i < ns; i++) {
        const int id = byte(), tables = byte();
        int which = -1;
        for (size_t k = 0; k < comp_.size(); k++)
            if (comp_[k].id == id) which = (int)k;
        if (which < 0) fail("Corrupt JPEG (bad SOS component)");
        comp_[which].hd = tables >> 4;
        comp_[which].ha = tables & 15;
        if (comp_[which].hd > 3 || comp_[which].ha > 3) fail("Corrupt JPEG (bad SOS tables)");
        scomp.push_back(which);
    }
    const int ss = byte(), se = byte(), ahal = byte();
    if (ss != 0 || se != 63 || ahal != 0) fail("Corrupt JPEG (bad SOS spectral selection)");
}

// One 8x8 block: Huffman DC/AC decode with inline dequantisation (products
// truncated to int16, as stored by stb), then the islow IDCT below.
void JpegDecoder::block(JComp& c, int16_t data[64]) {
    std::memset(data, 0, 64 * sizeof(int16_t));
    const Huffman& hd = hdc_[c.hd];
    const Huffman& ha = hac_[c.ha];
    if (!hd.defined || !ha.defined) fail("Corrupt JPEG (undefined Huffman table)");
    const uint16_t* dq = dq_[c.tq];
    const int t = huff(hd);
    if (t > 15) fail("Corrupt JPEG (bad huffman code)");
    const int diff = t ? extend(getbits(t), t) : 0;
    const long long dcl = (long long)c.dc_pred + diff;
    if (dcl > INT32_MAX || dcl < INT32_MIN) fail("Corrupt JPEG (bad delta)");
    const int dc = (int)dcl;
    c.dc_pred = dc;
    // stb's validity test for the product of two shorts (b = quantiser >= 0)
    const int b = dq[0];
    const bool ok = b == 0 || (dc >= 0 ? dc <= INT16_MAX / b : dc >= INT16_MIN / b);
    if (!ok) fail("Corrupt JPEG (can't merge dc and ac)");
    data[0] = (int16_t)(dc * b);
    int k = 1;
    do {
        const int rs = huff(ha);
        const int s = rs & 15, r = rs >> 4;
        if (s == 0) {
            if (rs != 0xF0) break;  // end of block
            k += 16;
        } else {
            k += r;
            const int zig = kDezigzag[k++];
            data[zig] = (int16_t)wmul(extend(getbits(s), s), dq[zig]);
        }
    } while (k < 64);
}

// islow IDCT (libjpeg jidctint), in 12-bit fixed point: columns keep two
// extra bits (>> 10 with +512), rows remove the rest (>> 17 with +2^16) and
// add the 128 level shift.  Intermediate products in int (wrapping as C int).
inline int fix12(double x) { return (int)(x * 4096 + 0.5); }

struct Idct1D {
    int t0, t1, t2, t3, x0, x1, x2, x3;
    void run(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
        // even part
        const int p1 = wmul(wadd(s2, s6), fix12(0.5411961f));
        const int e2 = wadd(p1, wmul(s6, fix12(-1.847759065f)));
        const int e3 = wadd(p1, wmul(s2, fix12(0.765366865f)));
        const int e0 = wmul(wadd(s0, s4), 4096);
        const int e1 = wmul(wsub(s0, s4), 4096);
        x0 = wadd(e0, e3);
        x3 = wsub(e0, e3);
        x1 = wadd(e1, e2);
        x2 = wsub(e1, e2);
        // odd part (s7, s5, s3, s1)
        int o0 = s7, o1 = s5, o2 = s3, o3 = s1;
        int q3 = wadd(o0, o2), q4 = wadd(o1, o3), q1 = wadd(o0, o3), q2 = wadd(o1, o2);
        const int q5 = wmul(wadd(q3, q4), fix12(1.175875602f));
        o0 = wmul(o0, fix12(0.298631336f));
        o1 = wmul(o1, fix12(2.053119869f));
        o2 = wmul(o2, fix12(3.072711026f));
        o3 = wmul(o3, fix12(1.501321110f));
        q1 = wadd(q5, wmul(q1, fix12(-0.899976223f)));
        q2 = wadd(q5, wmul(q2, fix12(-2.562915447f)));
        q3 = wmul(q3, fix12(-1.961570560f));
        q4 = wmul(q4, fix12(-0.390180644f));
        t3 = wadd(wadd(o3, q1), q4);
        t2 = wadd(wadd(o2, q2), q3);
        t1 = wadd(wadd(o1, q2), q4);
        t0 = wadd(wadd(o0, q1), q3);
    }
};

inline uint8_t clamp8(int x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); }

void idct_islow(const int16_t in[64], uint8_t* out, int stride) {
    int v[64];
    for (int i = 0; i < 8; i++) {
        const int16_t* d = in + i;
        Idct1D t;
        t.run(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56]);
        const int x0 = wadd(t.x0, 512), x1 = wadd(t.x1, 512), x2 = wadd(t.x2, 512), x3 = wadd(t.x3, 512);
        v[i + 0] = wadd(x0, t.t3) >> 10;
        v[i + 56] = wsub(x0, t.t3) >> 10;
        v[i + 8] = wadd(x1, t.t2) >> 10;
        v[i + 48] = wsub(x1, t.t2) >> 10;
        v[i + 16] = wadd(x2, t.t1) >> 10;
        v[i + 40] = wsub(x2, t.t1) >> 10;
        v[i + 24] = wadd(x3, t.t0) >> 10;
        v[i + 32] = wsub(x3, t.t0) >> 10;
    }
    for (int r = 0; r < 8; r++) {
        const int* s = v + 8 * r;
        uint8_t* o = out + (size_t)r * stride;
        Idct1D t;
        t.run(s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]);
        const int bias = 65536 + (128 << 17);
        const int x0 = wadd(t.x0, bias), x1 = wadd(t.x1, bias), x2 = wadd(t.x2, bias), x3 = wadd(t.x3, bias);
        o[0] = clamp8(wadd(x0, t.t3) >> 17);
        o[7] = clamp8(wsub(x0, t.t3) >> 17);
        o[1] = clamp8(wadd(x1, t.t2) >> 17);
        o[6] = clamp8(wsub(x1, t.t2) >> 17);
        o[2] = clamp8(wadd(x2, t.t1) >> 17);
        o[5] = clamp8(wsub(x2, t.t1) >> 17);
        o[3] = clamp8(wadd(x3, t.t0) >> 17);
        o[4] = clamp8(wsub(x3, t.t0) >> 17);
    }
}

void JpegDecoder::decode_scan(const std::vector<int>& scomp) {
    reset_bits();
    for (int c : scomp) comp_[c].dc_pred = 0;
    int16_t data[64];
    int todo = restart_ ? restart_ : 0x7fffffff;
    auto after_mcu = [&]() -> bool {  // false: stop the scan (marker that is not RSTn)
        if (--todo > 0) return true;
        if (bits_ < 24) fill();
        if (marker_ < 0xD0 || marker_ > 0xD7) return false;
        reset_bits();
        for (int c : scomp) comp_[c].dc_pred = 0;
        todo = restart_;
        return true;
    };
    if (scomp.size() == 1) {  // non-interleaved: the component's own block grid
        JComp& c = comp_[scomp[0]];
        const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
        for (int j = 0; j < bh; j++)
            for (int i = 0; i < bw; i++) {
                block(c, data);
                idct_islow(data, c.plane.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2);
                if (!after_mcu()) return;
            }
        return;
    }
    for (int my = 0; my < mcuy_; my++)
        for (int mx = 0; mx < mcux_; mx++) {
            for (int ci : scomp) {
                JComp& c = comp_[ci];
                for (int y = 0; y < c.v; y++)
                    for (int x = 0; x < c.h; x++) {
                        const int bx = (mx * c.h + x) * 8, by = (my * c.v + y) * 8;
                        block(c, data);
                        idct_islow(data, c.plane.data() + (size_t)c.w2 * by + bx, c.w2);
                    }
            }
            if (!after_mcu()) return;
        }
}

// stb's upsampling filters (jfif-centred), per output row
void up_h2(uint8_t* out, const uint8_t* in, int w) {
    if (w == 1) {
        out[0] = out[1] = in[0];
        return;
    }
    out[0] = in[0];
    out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
    int i;
    for (i = 1; i < w - 1; ++i) {
        const int n = 3 * in[i] + 2;
        out[i * 2] = (uint8_t)((n + in[i - 1]) >> 2);
        out[i * 2 + 1] = (uint8_t)((n + in[i + 1]) >> 2);
    }
    out[i * 2] = (uint8_t)((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
    out[i * 2 + 1] = in[w - 1];
}
void up_v2(uint8_t* out, const uint8_t* nr, const uint8_t* fr, int w) {
    for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * nr[i] + fr[i] + 2) >> 2);
}
void up_hv2(uint8_t* out, const uint8_t* nr, const uint8_t* fr, int w) {
    if (w == 1) {
        out[0] = out[1] = (uint8_t)((3 * nr[0] + fr[0] + 2) >> 2);
        return;
    }
    int t1 = 3 * nr[0] + fr[0];
    out[0] = (uint8_t)((t1 + 2) >> 2);
    for (int i = 1; i < w; ++i) {
        const int t0 = t1;
        t1 = 3 * nr[i] + fr[i];
        out[i * 2 - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
        out[i * 2] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
    }
    out[w * 2 - 1] = (uint8_t)((t1 + 2) >> 2);
}
void up_nearest(uint8_t* out, const uint8_t* in, int w, int hs) {
    for (int i = 0; i < w; ++i)
        for (int j = 0; j < hs; ++j) out[i * hs + j] = in[i];
}

// stb's reduced-precision fixed-point YCbCr -> RGB
inline int ycc_fix(float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; }
void ycc_to_rgb(uint8_t* out, const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int count, int step) {
    for (int i = 0; i < count; ++i) {
        const int yf = (y[i] << 20) + (1 << 19);
        const int vr = cr[i] - 128, vb = cb[i] - 128;
        int r = yf + vr * ycc_fix(1.40200f);
        int g = yf + (vr * -ycc_fix(0.71414f)) + ((vb * -ycc_fix(0.34414f)) & (int)0xffff0000u);
        int b = yf + vb * ycc_fix(1.77200f);
        r >>= 20;
        g >>= 20;
        b >>= 20;
        out[0] = clamp8(r);
        out[1] = clamp8(g);
        out[2] = clamp8(b);
        out += step;
    }
}

Image JpegDecoder::decode() {
    if (d_.size() < 2 || d_[0] != 0xFF || d_[1] != 0xD8) fail("not a JPEG");
    pos_ = 2;
    bool have_sof = false, done = false;
    while (!done) {
        const int m = next_marker();
        if (m == 0xD9) break;                       // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;       // stray RSTn
        if (m == 0x01) continue;                    // TEM
        const int len = word();
        if (len < 2) fail("Corrupt JPEG (bad marker length)");
        const size_t seg_end = pos_ + len - 2;
        if (seg_end > d_.size()) fail("Corrupt JPEG (truncated segment)");
        switch (m) {
        case 0xDB: read_dqt(len); break;
        case 0xC4: read_dht(len); break;
        case 0xDD:
            if (len != 4) fail("Corrupt JPEG (bad DRI len)");
            restart_ = word();
            break;
        case 0xC0:
        case 0xC1:
            if (have_sof) fail("Corrupt JPEG (multiple SOF)");
            read_sof(len);
            have_sof = true;
            break;
        case 0xC2:
            fail("JPEG: progressive JPEG is not supported");
        case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
        case 0xCD: case 0xCE: case 0xCF:
            fail("JPEG: only sequential Huffman JPEG is supported");
        case 0xDA: {
            if (!have_sof) fail("Corrupt JPEG (SOS before SOF)");
            std::vector<int> sc;
            read_sos(len, sc);
            decode_scan(sc);
            // continue after the entropy-coded segment: at the marker that ended it
            if (marker_ >= 0) pos_ -= 2;
            if (marker_ < 0) {
                // scan ended by MCU count: resync on the next marker
            }
            continue;
        }
        case 0xE0:  // APP0: JFIF
            if (len >= 7 && std::memcmp(&d_[pos_], "JFIF\0", 5) == 0) jfif_ = true;
            pos_ = seg_end;
            break;
        case 0xEE:  // APP14: Adobe, colour transform flag
            if (len >= 14 && std::memcmp(&d_[pos_], "Adobe", 5) == 0) app14_ = d_[pos_ + 11];
            pos_ = seg_end;
            break;
        default:
            pos_ = seg_end;  // APPn, COM, ...
            break;
        }
    }
    if (!have_sof) fail("Corrupt JPEG (no SOF)");

    const int nc = (int)comp_.size();
    const int n = nc >= 3 ? 3 : 1;
    int rgb_ids = 0;
    if (nc == 3) {
        static const int ids[3] = {'R', 'G', 'B'};
        for (int i = 0; i < 3; i++) rgb_ids += comp_[i].id == ids[i];
    }
    const bool is_rgb = nc == 3 && (rgb_ids == 3 || (app14_ == 0 && !jfif_));
    struct Res {
        int hs, vs, ystep, w_lo, ypos;
        const uint8_t *line0, *line1;
        std::vector<uint8_t> buf;
    };
    std::vector<Res> rs(nc);
    for (int k = 0; k < nc; k++) {
        Res& r = rs[k];
        r.hs = hmax_ / comp_[k].h;
        r.vs = vmax_ / comp_[k].v;
        r.ystep = r.vs >> 1;
        r.w_lo = (w_ + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = comp_[k].plane.data();
        r.buf.assign((size_t)w_ + 3, 0);
    }
    Image im;
    im.w = w_;
    im.h = h_;
    im.n = n;
    im.px.assign((size_t)w_ * h_ * n, 0);
    std::vector<const uint8_t*> co(nc);
    for (int j = 0; j < h_; j++) {
        uint8_t* out = im.px.data() + (size_t)n * w_ * j;
        for (int k = 0; k < nc; k++) {
            Res& r = rs[k];
            const bool y_bot = r.ystep >= (r.vs >> 1);
            const uint8_t* nr = y_bot ? r.line1 : r.line0;
            const uint8_t* fr = y_bot ? r.line0 : r.line1;
            if (r.hs == 1 && r.vs == 1) {
                co[k] = nr;
            } else if (r.hs == 1 && r.vs == 2) {
                up_v2(r.buf.data(), nr, fr, r.w_lo);
                co[k] = r.buf.data();
            } else if (r.hs == 2 && r.vs == 1) {
                up_h2(r.buf.data(), nr, r.w_lo);
                co[k] = r.buf.data();
            } else if (r.hs == 2 && r.vs == 2) {
                up_hv2(r.buf.data(), nr, fr, r.w_lo);
                co[k] = r.buf.data();
            } else {
                if ((size_t)r.w_lo * r.hs > r.buf.size()) r.buf.resize((size_t)r.w_lo * r.hs);
                up_nearest(r.buf.data(), nr, r.w_lo, r.hs);
                co[k] = r.buf.data();
            }
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < comp_[k].y) r.line1 += comp_[k].w2;
            }
        }
        if (n == 3) {
            if (is_rgb) {
                for (int i = 0; i < w_; i++) {
                    out[3 * i] = co[0][i];
                    out[3 * i + 1] = co[1][i];
                    out[3 * i + 2] = co[2][i];
                }
            } else {
                ycc_to_rgb(out, co[0], co[1], co[2], w_, 3);
            }
        } else {
            std::memcpy(out, co[0], (size_t)w_);
        }
    }
    return im;
}

void flip_rows(Image& im) {
    const size_t row = (size_t)im.w * im.n;
    std::vector<uint8_t> tmp(row);
    for (int y = 0; y < im.h / 2; y++) {
        uint8_t* a = im.px.data() + row * y;
        uint8_t* b = im.px.data() + row * (im.h - 1 - y);
        std::memcpy(tmp.data(), a, row);
        std::memcpy(a, b, row);
        std::memcpy(b, tmp.data(), row);
    }
}

}  // namespace

Image load_image(const std::string& path, bool flip) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open image " + path);
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    Image im;
    try {
        if (d.size() >= 8 && d[0] == 137 && d[1] == 'P' && d[2] == 'N' && d[3] == 'G')
            im = decode_png(d);
        else if (d.size() >= 2 && d[0] == 0xFF && d[1] == 0xD8)
            im = JpegDecoder(d).decode();
        else
            fail("unknown image type");
    } catch (const Fail& e) {
        throw std::runtime_error(path + ": " + e.what());
    }
    if (flip) flip_rows(im);
    return im;
}

}  // namespace rt2h

extern "C" int rt2_image_load(const char* path, int32_t flip_vertically, rt2_image* out) {
    return rt2h::guard([&]() -> int {
        if (!path || !out) throw std::runtime_error("null argument");
        rt2h::Image im = rt2h::load_image(path, flip_vertically != 0);
        uint8_t* px = (uint8_t*)std::malloc(im.px.size() ? im.px.size() : 1);
        if (!px) throw std::runtime_error("out of memory");
        std::memcpy(px, im.px.data(), im.px.size());
        out->width = im.w;
        out->height = im.h;
        out->channels = im.n;
        out->pixels = px;
        return 0;
    });
}

extern "C" void rt2_image_free(rt2_image* img) {
    if (!img) return;
    std::free(img->pixels);
    img->pixels = nullptr;
}
