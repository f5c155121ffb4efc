// OBJ/MTL loader: restatement of getTrianglesData_ (RayTracing/Assets/headers/
// mesh.h:279-613) behind rt2_sd_load_obj_folder.  Semantics kept on purpose,
// because they decide the arrays the render path consumes:
//   - the OBJ is the first *.obj of the folder in directory order (:223-253);
//   - textures: the regular files of <folder>/textures in directory order give
//     the texture indices (:305-318); each is decoded (image.cpp) and kept;
//   - every folder file whose text after its FIRST '.' is "mtl" is parsed, in
//     directory order; a folder file with no '.' is an error (:328-339);
//   - material `index` = running count of `newmtl` over all MTL files (:369),
//     and that index is what a triangle stores (:602);
//   - the material ARRAY is "_default_" plus every library, flattened in
//     std::map (byte-string) order of library name then material name
//     (:456-462) — so array position and `index` differ when names are not
//     already sorted, exactly as in the reference;
//   - Ke > 0 makes a LIGHT of strength 0.299 r + 0.587 g + 0.114 b (:378-398);
//   - faces must have exactly three ' ' characters (:501-506); UVs are stored
//     in the order (t1, t2, t0) (:602-606).
#include <algorithm>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>

#include "host_internal.h"

namespace fs = std::filesystem;
using namespace rt2h;

namespace {

// getFilenamesInFolder, external/filesUtil/myFile.cpp:67-85
std::vector<std::string> filenames_in(const fs::path& folder) {
    std::vector<std::string> out;
    std::error_code ec;
    if (fs::exists(folder, ec) && fs::is_directory(folder, ec)) {
        for (const auto& e : fs::directory_iterator(folder)) {
            if (fs::is_regular_file(e.status())) out.push_back(e.path().filename().string());
        }
    }
    return out;
}

// findFirstObjFile, mesh.h:223-253
fs::path first_obj(const fs::path& folder) {
    std::error_code ec;
    if (!fs::exists(folder, ec) || !fs::is_directory(folder, ec)) return fs::path();
    for (const auto& e : fs::directory_iterator(folder)) {
        if (e.is_regular_file() && e.path().extension() == ".obj") return e.path();
    }
    return fs::path();
}

// split(str, ' '), mesh.h:156-175 (empty tokens dropped)
std::vector<std::string> split_ws(const std::string& s) {
    std::vector<std::string> r;
    std::string tok;
    for (char ch : s) {
        if (ch == ' ') {
            if (!tok.empty()) {
                r.push_back(tok);
                tok.clear();
            }
        } else {
            tok += ch;
        }
    }
    if (!tok.empty()) r.push_back(tok);
    return r;
}

rt2_material default_material() {
    rt2_material m;
    rt2_material_default(&m);
    return m;
}

int to_index(const std::string& s, size_t n, const std::string& line) {
    int i = std::stoi(s) - 1;  // 1-based, as mesh.h:523
    if (i < 0 || (size_t)i >= n) throw std::runtime_error("OBJ index out of range in line: " + line);
    return i;
}

}  // namespace

extern "C" int rt2_sd_load_obj_folder(rt2_scene_data* sd, const char* folder_c) {
    return guard([&]() -> int {
        if (!sd || !folder_c) throw std::runtime_error("null argument");
        fs::path obj = first_obj(folder_c);
        if (obj.empty()) throw std::runtime_error(std::string("OBJ file not found in ") + folder_c);
        fs::path folder = obj.parent_path();
        std::ifstream objs(obj);
        if (!objs.is_open()) throw std::runtime_error("cannot open " + obj.string());

        // Textures (mesh.h:305-318): every file of textures/, in directory
        // order, decoded as Texture2D(path) does (textureClass.cpp:55-68:
        // flipped on load; a file stb cannot load throws).  Indices restart at
        // 0 for each folder, as the reference's per-call texture vector.
        std::map<std::string, int> tex_index;
        std::vector<std::string> tex = filenames_in(folder / "textures");
        for (size_t i = 0; i < tex.size(); i++) {
            tex_index[tex[i]] = (int)i;
            sd->textures.push_back(load_image((folder / "textures" / tex[i]).string(), true));
            sd->tex_names.push_back(tex[i]);
        }

        // MTL libraries (mesh.h:321-453).
        std::map<std::string, std::map<std::string, rt2_material>> libs;
        {
            rt2_material d = default_material();
            d.index = 0;
            libs["_default_"]["_default_"] = d;
        }
        int mat_index = 0;
        for (const std::string& name : filenames_in(folder)) {
            size_t dot = name.find('.');
            if (dot == std::string::npos) throw std::runtime_error("File extension not found: " + name);
            if (name.substr(dot + 1) != "mtl") continue;
            std::ifstream ms(folder / name);
            if (!ms.is_open()) continue;
            std::map<std::string, rt2_material> by_name;
            std::string mtl_name;
            while (!ms.eof()) {
                char line[256];
                ms.getline(line, 256);
                if (ms.fail() && !ms.eof())
                    throw std::runtime_error("MTL line longer than 255 characters in " + name +
                                             " (the reference's getline loop never terminates on it)");
                std::stringstream ss;
                ss << line;
                std::string key;
                ss >> key;
                if (key == "newmtl") {
                    ss >> mtl_name;
                    rt2_material m = default_material();
                    m.index = ++mat_index;
                    by_name[mtl_name] = m;
                } else if (key == "Kd") {
                    float v[3] = {0.0f, 0.0f, 0.0f};
                    ss >> v[0] >> v[1] >> v[2];
                    rt2_material& m = by_name[mtl_name];
                    m.color = rt2_vec4{v[0], v[1], v[2], 0.0f};
                } else if (key == "Ke") {
                    float v[3] = {0.0f, 0.0f, 0.0f};
                    ss >> v[0] >> v[1] >> v[2];
                    rt2_material& m = by_name[mtl_name];
                    if (v[0] > 0.0f || v[1] > 0.0f || v[2] > 0.0f) {
                        float strength = 0.299f * v[0] + 0.587f * v[1] + 0.114f * v[2];
                        rt2_material_make_light(&m, v[0], v[1], v[2], strength);
                    } else {
                        m.emissionColor = rt2_vec4{v[0], v[1], v[2], 0.0f};
                        m.emissionStrength = 0.0f;
                    }
                } else if (key == "GlassHighlight") {
                    rt2_material& m = by_name[mtl_name];
                    if (m.materialType != RT2_LIGHT) {  // makeGlassHighlight, mesh.h:92-96
                        m.materialType = RT2_GLASS_HIGHLIGHT;
                        m.color.w = 0.0f;
                    }
                } else if (key == "EDGE_HIGHLIGHT") {
                    by_name[mtl_name].isEdgeHighlight = 1;
                } else if (key == "map_Kd") {
                    rt2_material& m = by_name[mtl_name];
                    if (m.materialType != RT2_LIGHT && m.materialType != RT2_GLASS &&
                        m.materialType != RT2_GLASS_HIGHLIGHT) {
                        std::string tex_name;
                        ss >> tex_name;
                        m.materialType = RT2_TEXTURE;
                        auto it = tex_index.find(tex_name);
                        if (it == tex_index.end())
                            throw std::runtime_error("texture not found in textures/: " + tex_name);
                        m.textureIndex = it->second;
                    }
                }
            }
            libs[name] = by_name;
        }
        for (const auto& lib : libs)
            for (const auto& kv : lib.second) sd->mats.push_back(kv.second);

        // OBJ (mesh.h:465-610).
        std::vector<V3> verts;
        std::vector<float> uvs;  // pairs
        std::string cur_lib = "_default_", cur_mtl = "_default_";
        std::string line;
        while (!objs.eof()) {
            std::getline(objs, line);
            std::stringstream ss(line);
            std::string type;
            ss >> type;
            if (type == "mtllib") {
                ss >> cur_lib;
            } else if (type == "usemtl") {
                ss >> cur_mtl;
            } else if (type == "v") {
                V3 v;
                ss >> v.x >> v.y >> v.z;
                verts.push_back(v);
            } else if (type == "vt") {
                float a = 0.0f, b = 0.0f;
                ss >> a >> b;
                uvs.push_back(a);
                uvs.push_back(b);
            } else if (type == "f") {
                if (std::count(line.begin(), line.end(), ' ') != 3)
                    throw std::runtime_error("Invalid OBJ file, non-triangle face not supported. Line: " + line);
                std::vector<std::string> fd = split_ws(line);
                if (fd.size() < 2) throw std::runtime_error("malformed face: " + line);
                int slashes = (int)std::count(fd[1].begin(), fd[1].end(), '/');
                V3 p[3];
                float uv[3][2] = {{0, 0}, {0, 0}, {0, 0}};
                const size_t nuv = uvs.size() / 2;
                for (int i = 0; i < 3; i++) {
                    std::string tok;
                    ss >> tok;
                    size_t s1 = tok.find('/');
                    if (slashes == 0) {
                        p[i] = verts[to_index(tok, verts.size(), line)];
                    } else if (slashes == 1) {
                        p[i] = verts[to_index(tok.substr(0, s1), verts.size(), line)];
                        int t = to_index(tok.substr(s1 + 1), nuv, line);
                        uv[i][0] = uvs[2 * t];
                        uv[i][1] = uvs[2 * t + 1];
                    } else if (slashes == 2 && fd[1].find("//") == std::string::npos) {
                        p[i] = verts[to_index(tok.substr(0, s1), verts.size(), line)];
                        size_t s2 = tok.find('/', s1 + 1);
                        int t = to_index(tok.substr(s1 + 1, s2 - s1 - 1), nuv, line);
                        uv[i][0] = uvs[2 * t];
                        uv[i][1] = uvs[2 * t + 1];
                    } else {  // v//vn and the fallback of :572-589
                        p[i] = verts[to_index(s1 != std::string::npos ? tok.substr(0, s1) : tok, verts.size(), line)];
                    }
                }
                auto lib = libs.find(cur_lib);
                if (lib == libs.end() || lib->second.find(cur_mtl) == lib->second.end())
                    throw std::runtime_error("Requested material or library not found: " + cur_lib + ", " + cur_mtl);
                const rt2_material& m = lib->second.at(cur_mtl);
                rt2_triangle t{};
                t.a = vec4(p[0]);
                t.b = vec4(p[1]);
                t.c = vec4(p[2]);
                t.aTex = rt2_vec2{uv[1][0], uv[1][1]};
                t.bTex = rt2_vec2{uv[2][0], uv[2][1]};
                t.cTex = rt2_vec2{uv[0][0], uv[0][1]};
                t.materialIndex = m.index;
                sd->push(t);
            }
        }
        return 0;
    });
}
