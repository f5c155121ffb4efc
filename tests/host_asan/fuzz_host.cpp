// Host-side robustness check under AddressSanitizer + UBSan (CPU only; the
// GPU path is not involved).  Decodes every golden image, then thousands of
// corrupted variants (truncations, bit flips, byte stores, chunk-length
// damage): each must either decode or fail with an error — never read or
// write out of bounds.  Also loads OBJ folders given on the command line.
//
//   make -C tests/host_asan && tests/host_asan/fuzz_host tests/golden/images/*
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt2.h"

static std::vector<unsigned char> slurp(const char* p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static int decode_bytes(const std::vector<unsigned char>& d, const char* tmp) {
    {
        std::ofstream o(tmp, std::ios::binary);
        o.write((const char*)d.data(), (std::streamsize)d.size());
    }
    rt2_image im;
    const int rc = rt2_image_load(tmp, 1, &im);
    if (rc == 0) {
        volatile unsigned s = 0;  // touch every byte
        for (size_t i = 0; i < (size_t)im.width * im.height * im.channels; i++) s += im.pixels[i];
        rt2_image_free(&im);
    }
    return rc;
}

int main(int argc, char** argv) {
    const char* tmp = "/tmp/rt2_fuzz_image.bin";
    std::mt19937 rng(12345);
    int ok = 0, failed = 0, cases = 0;
    for (int a = 1; a < argc; a++) {
        const std::vector<unsigned char> src = slurp(argv[a]);
        if (src.empty()) continue;
        if (decode_bytes(src, tmp) != 0)  // e.g. progressive JPEG (rejected by design): fuzz it anyway
            std::printf("note: %s does not decode: %s\n", argv[a], rt2_last_error());
        for (int k = 0; k < 400; k++) {
            std::vector<unsigned char> d = src;
            const int kind = k % 5;
            const size_t n = d.size();
            if (kind == 0) {
                d.resize(std::uniform_int_distribution<size_t>(0, n)(rng));
            } else if (kind == 1) {
                for (int f = 0; f < 1 + (int)(rng() % 8); f++) d[rng() % n] ^= (unsigned char)(1u << (rng() % 8));
            } else if (kind == 2) {
                for (int f = 0; f < 1 + (int)(rng() % 4); f++) d[rng() % n] = (unsigned char)rng();
            } else if (kind == 3) {
                const size_t at = rng() % n;  // 0xFF runs (JPEG markers) / large lengths (PNG)
                for (size_t i = at; i < std::min(n, at + 4); i++) d[i] = 0xFF;
            } else {
                const size_t at = std::min<size_t>(8 + (rng() % 64), n ? n - 1 : 0);
                for (size_t i = at; i < std::min(n, at + 4); i++) d[i] = (unsigned char)(rng() & 1 ? 0 : 0x7f);
            }
            (decode_bytes(d, tmp) == 0 ? ok : failed)++;
            cases++;
        }
    }
    std::printf("fuzzed %d corrupted images: %d decoded, %d rejected with an error\n", cases, ok, failed);

    // OBJ/MTL loader on corrupted text (mesh.h:279-613 restatement)
    const std::string base_obj =
        "mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvt 0 0\nvt 1 0\nvt 0 1\nvn 0 0 1\n"
        "usemtl A\nf 1/1/1 2/2/1 3/3/1\nusemtl B\nf 2/2/1 4/1/1 3/3/1\n";
    const std::string base_mtl =
        "newmtl A\nKd 0.8 0.2 0.2\nKe 0 0 0\nnewmtl B\nKd 0.1 0.9 0.1\nKe 1 1 1\nNi 1.5\nd 0.5\n";
    const std::string dir = "/tmp/rt2_fuzz_obj";
    std::system(("rm -rf " + dir + " && mkdir -p " + dir).c_str());
    const char alphabet[] = " /\n0123456789.-eEfvntu#";
    int lok = 0, lfail = 0;
    for (int k = 0; k < 3000; k++) {
        std::string obj = base_obj, mtl = base_mtl;
        std::string& t = (k & 1) ? obj : mtl;
        for (int f = 0; f < 1 + (int)(rng() % 6); f++) {
            const size_t at = rng() % t.size();
            switch (rng() % 3) {
            case 0: t[at] = alphabet[rng() % (sizeof(alphabet) - 1)]; break;
            case 1: t.erase(at, 1 + rng() % 5); break;
            default: t.insert(at, std::string(1 + rng() % 3, alphabet[rng() % (sizeof(alphabet) - 1)])); break;
            }
            if (t.empty()) t = "v 0 0 0\n";
        }
        std::ofstream(dir + "/m.obj") << obj;
        std::ofstream(dir + "/m.mtl") << mtl;
        rt2_scene_data* sd = rt2_sd_create();
        (rt2_sd_load_obj_folder(sd, dir.c_str()) == 0 ? lok : lfail)++;
        if (rt2_sd_num_triangles(sd) > 0) rt2_sd_build_bvh(sd);
        rt2_sd_destroy(sd);
    }
    std::printf("fuzzed 3000 corrupted OBJ/MTL folders: %d loaded, %d rejected with an error\n", lok, lfail);
    return 0;
}
