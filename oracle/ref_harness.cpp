// TEST INFRASTRUCTURE ONLY.  Drives the reference's own host code, compiled
// from /root/reference where it lies (see Makefile target `ref`), to dump
// golden fixtures for the host surface of the render path:
//   - Camera(...) + updateUniforms         camera.h:99-192
//   - the scene builders                   rayTracing.cpp:388-1118
//   - BVH(bvhTriangles, rtxTriangles)      BVH.h:145-221 (node array + reorder)
//   - Material constructors                mesh.h:47-102
// The GLSL kernel itself cannot run here; the OBJ loader
// cannot link without a stand-in for filesUtil/myFile.cpp's <windows.h>, so it
// is not driven (its parity is pinned by tests/test_host_loader.py instead).
//
// Protocol: ref_dump <command> <in> <out> [args].  All files are raw
// little-endian arrays of the reference structs.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

#include "RayTracing/src/rayTracing.cpp"

static std::vector<RTXTriangle> read_tris(const char* path) {
    std::vector<RTXTriangle> out;
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    RTXTriangle t(0, glm::vec4(0), glm::vec4(0), glm::vec4(0), glm::vec2(0), glm::vec2(0), glm::vec2(0));
    static_assert(sizeof(RTXTriangle) == 80, "RTXTriangle layout");
    while (std::fread(&t, sizeof(t), 1, f) == 1) out.push_back(t);
    std::fclose(f);
    return out;
}

static std::vector<BVHTriangle> bvh_tris_of(const std::vector<RTXTriangle>& r) {
    std::vector<BVHTriangle> b;
    for (const RTXTriangle& t : r) b.push_back(BVHTriangle(glm::vec3(t.a), glm::vec3(t.b), glm::vec3(t.c)));
    return b;
}

static void put_i32(FILE* f, int32_t v) { std::fwrite(&v, 4, 1, f); }

static void put_scene(FILE* f, const std::vector<RTXTriangle>& r, const std::vector<BVHTriangle>& b) {
    put_i32(f, (int32_t)r.size());
    std::fwrite(r.data(), sizeof(RTXTriangle), r.size(), f);
    for (const BVHTriangle& t : b) {
        float v[9] = {t.min.x, t.min.y, t.min.z, t.max.x, t.max.y, t.max.z, t.center.x, t.center.y, t.center.z};
        std::fwrite(v, 4, 9, f);
    }
}

int harness_main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: ref_dump camera|builders|bvh|materials <in> <out> [W H]\n");
        return 2;
    }
    std::string cmd = argv[1];
    // The reference prints progress on stdout; keep stdout for it, data goes to files.
    if (cmd == "camera") {
        int W = std::atoi(argv[4]), H = std::atoi(argv[5]);
        // rayTracing.cpp:1337 with the globals of :82-89
        Camera camera(W, H, maxSpeed, cameraPos, hfov, pitch, yaw, focusDistance, defocusAngle, zoom);
        GlobalUniforms u;
        std::memset(&u, 0, sizeof(u));
        camera.updateUniforms(u);
        static_assert(sizeof(GlobalUniforms) == 192, "GlobalUniforms layout");
        FILE* f = std::fopen(argv[3], "wb");
        std::fwrite(&u, sizeof(u), 1, f);
        std::fclose(f);
        return 0;
    }
    if (cmd == "materials") {
        // mesh.h constructors as main() uses them (rayTracing.cpp:1268-1283).
        std::vector<Material> m(7);
        m[0] = Material();
        m[1].makeDiffusive(glm::vec3(1.0f, 0.0f, 0.0f));
        m[2].makeLight(glm::vec3(1.0f), CORNELL_LIGHT_BRIGHTNESS);
        m[3].makeSpecular(glm::vec3(1.0f), glm::vec3(1.0f), 1.0f, 1.0f);
        m[4].makeChecker(4.0f);
        m[5].makeGlass(glm::vec3(0.9f, 0.8f, 0.7f), 1.5f);
        m[6].makeGlassHighlight(glm::vec3(0.25f, 0.5f, 0.75f));
        static_assert(sizeof(Material) == 96, "Material layout");
        FILE* f = std::fopen(argv[3], "wb");
        std::fwrite(m.data(), sizeof(Material), m.size(), f);
        std::fclose(f);
        return 0;
    }
    if (cmd == "builders") {
        std::vector<RTXTriangle> base = read_tris(argv[2]);
        FILE* f = std::fopen(argv[3], "wb");
        // Material indices follow main(): base materials then red, green, wall, light, mirror.
        const int red = 100, green = 101, white = 102, light = 103, mirror = 104;
        {   // addCornellBox(rtx, bvh, CORNELL_LIGHT_SIZE, CORNELL_PADDING, light, true)  :453
            std::vector<RTXTriangle> r = base;
            std::vector<BVHTriangle> b = bvh_tris_of(r);
            addCornellBox(r, b, CORNELL_LIGHT_SIZE, CORNELL_PADDING, light, true);
            put_scene(f, r, b);
        }
        {   // addMirrorCornellBox  :569
            std::vector<RTXTriangle> r = base;
            std::vector<BVHTriangle> b = bvh_tris_of(r);
            addMirrorCornellBox(r, b, CORNELL_LIGHT_SIZE, CORNELL_PADDING, light, mirror);
            put_scene(f, r, b);
        }
        {   // addSideLitCornellBox, both orientations  :690
            for (int rot = 0; rot < 2; rot++) {
                std::vector<RTXTriangle> r = base;
                std::vector<BVHTriangle> b = bvh_tris_of(r);
                addSideLitCornellBox(r, b, CORNELL_LIGHT_SIZE, CORNELL_PADDING, light, white, rot);
                put_scene(f, r, b);
            }
        }
        {   // addSkyLightPlane  :388
            std::vector<RTXTriangle> r = base;
            std::vector<BVHTriangle> b = bvh_tris_of(r);
            addSkyLightPlane(r, b, light);
            put_scene(f, r, b);
        }
        {   // createClassicCornellBox(…, 10, …)  :949
            std::vector<RTXTriangle> r;
            std::vector<BVHTriangle> b;
            createClassicCornellBox(r, b, 10.0f, red, green, white, light);
            put_scene(f, r, b);
        }
        {   // createDiverseCornellBox  :1071
            std::vector<RTXTriangle> r;
            std::vector<BVHTriangle> b;
            createDiverseCornellBox(r, b, 10.0f, red, green, white, light, 105, mirror, 106, 107);
            put_scene(f, r, b);
        }
        std::fclose(f);
        return 0;
    }
    if (cmd == "bvh") {
        // BVH over the triangles as given; BVH triangles from each triangle's
        // own vertices (mesh.h:608; for addCornellBox this is the corrected
        // light table, SURVEY.md §7 "Reference UB").
        std::vector<RTXTriangle> r = read_tris(argv[2]);
        std::vector<BVHTriangle> b = bvh_tris_of(r);
        std::streambuf* old = std::cout.rdbuf();
        std::ofstream devnull("/dev/null");
        std::cout.rdbuf(devnull.rdbuf());  // BVH::split prints every leaf (BVH.h:213-219)
        BVH bvh(b, r);
        std::cout.rdbuf(old);
        static_assert(sizeof(Node) == 48, "Node layout");
        FILE* f = std::fopen(argv[3], "wb");
        put_i32(f, (int32_t)bvh.allNodes.size());
        std::fwrite(bvh.allNodes.data(), sizeof(Node), bvh.allNodes.size(), f);
        put_i32(f, (int32_t)r.size());
        std::fwrite(r.data(), sizeof(RTXTriangle), r.size(), f);
        std::fclose(f);
        return 0;
    }
    std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 2;
}
