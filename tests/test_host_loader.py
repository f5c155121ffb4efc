"""OBJ/MTL loader semantics of getTrianglesData_ (mesh.h:279-613).

The reference loader cannot be linked here without a stand-in for
filesUtil/myFile.cpp's <windows.h> (tests/golden/make_golden.py), so its
behaviour is pinned by (a) the reference's own model files with hand-derived
expectations and (b) synthetic folders exercising each rule of mesh.h.
"""
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, needs_reference

DATA = "/root/reference/RayTracing/Data"


def write(folder, name, text):
    os.makedirs(folder, exist_ok=True)
    with open(os.path.join(folder, name), "w") as f:
        f.write(text)


def load(rt2mod, folder):
    sd = rt2mod.SceneData()
    sd.load_obj_folder(str(folder))
    return sd


@needs_reference
def test_campfire_counts_and_lights(rt2mod):
    sd = load(rt2mod, os.path.join(DATA, "campfire"))
    assert sd.num_triangles == 1192
    m = sd.materials()
    assert len(m) == 7
    assert m[0]["index"] == 0 and m[0]["materialType"] == rt2mod.DIFFUSE
    assert list(m["index"]) == list(range(7))  # names already sorted in campfire.mtl
    lights = np.nonzero(m["materialType"] == rt2mod.LIGHT)[0]
    assert list(lights) == [4, 6]
    # Ke 3 0.285921 0.047988 -> 0.299*3 + 0.587*0.285921 + 0.114*0.047988 (float arithmetic)
    f = np.float32
    s4 = f(f(f(0.299) * f(3.0)) + f(f(0.587) * f(0.285921))) + f(f(0.114) * f(0.047988))
    assert m[4]["emissionStrength"] == s4
    assert abs(m[6]["emissionStrength"] - 2.37494) < 1e-5
    assert np.allclose(m[1]["color"][:3], [0.187821, 0.278894, 0.332452])


@needs_reference
@pytest.mark.parametrize("model", ["campfire", "windmill", "cat"])
def test_model_fixture_matches_loader(rt2mod, model):
    """The loader-output fixtures the GPU box builds configs B/D, W and K from
    (tests/golden/make_golden.py, make_models.py) equal the loader's output on
    the reference's model files."""
    sd = load(rt2mod, os.path.join(DATA, model))
    z = np.load(os.path.join(GOLDEN, f"{model}_loaded.npz"), allow_pickle=False)
    assert sd.triangles().tobytes() == z["triangles"].tobytes()
    assert sd.materials().tobytes() == z["materials"].tobytes()


@needs_reference
@pytest.mark.parametrize("model,count", [("cat", 2832), ("windmill", 1805), ("sleeping", 372), ("building", 35385)])
def test_reference_models_load(rt2mod, model, count):
    sd = load(rt2mod, os.path.join(DATA, model))
    assert sd.num_triangles == count
    assert np.all(sd.triangles()["materialIndex"] >= 0)


def test_material_index_vs_array_order(rt2mod, tmp_path):
    """index = running newmtl count in directory order (mesh.h:369); array = std::map order (:456-462)."""
    d = tmp_path / "m"
    write(d, "zz.mtl", "newmtl Zeta\nKd 0.1 0.2 0.3\nnewmtl Alpha\nKd 0.4 0.5 0.6\n")
    write(d, "aa.mtl", "newmtl Mid\nKd 0.7 0.8 0.9\n")
    write(d, "model.obj", "mtllib zz.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl Zeta\nf 1 2 3\nusemtl Alpha\nf 1 3 2\n"
                          "mtllib aa.mtl\nusemtl Mid\nf 2 3 1\n")
    sd = load(rt2mod, d)
    files = [f for f in os.listdir(d) if os.path.isfile(os.path.join(d, f))]  # directory_iterator order
    order = {}
    k = 0
    for f in files:
        if f.split(".", 1)[1] == "mtl":
            for line in open(os.path.join(d, f)):
                if line.startswith("newmtl"):
                    k += 1
                    order[(f, line.split()[1])] = k
    m = sd.materials()
    # array: _default_ then aa.mtl{Mid} then zz.mtl{Alpha, Zeta}  (byte-string map order)
    assert list(m["index"]) == [0, order[("aa.mtl", "Mid")], order[("zz.mtl", "Alpha")], order[("zz.mtl", "Zeta")]]
    t = sd.triangles()
    assert list(t["materialIndex"]) == [order[("zz.mtl", "Zeta")], order[("zz.mtl", "Alpha")],
                                        order[("aa.mtl", "Mid")]]


def test_face_formats_and_uv_permutation(rt2mod, tmp_path):
    d = tmp_path / "f"
    write(d, "x.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0.1 0.2\nvt 0.3 0.4\nvt 0.5 0.6\nvn 0 0 1\n"
                      "f 1/1 2/2 3/3\nf 1/1/1 2/2/1 3/3/1\nf 1//1 2//1 3//1\nf 3 2 1\n")
    sd = load(rt2mod, d)
    t = sd.triangles()
    assert len(t) == 4
    for i in range(3):
        assert np.array_equal(t[i]["a"][:3], [0, 0, 0]) and np.array_equal(t[i]["c"][:3], [0, 1, 0])
    # RTXTriangle(…, tex[1], tex[2], tex[0]) (mesh.h:602-606)
    for i in (0, 1):
        assert np.allclose(t[i]["aTex"], [0.3, 0.4]) and np.allclose(t[i]["bTex"], [0.5, 0.6])
        assert np.allclose(t[i]["cTex"], [0.1, 0.2])
    assert np.array_equal(t[3]["a"][:3], [0, 1, 0])
    assert np.all(t["materialIndex"] == 0)  # no mtllib/usemtl -> _default_


def test_light_emission_glass_highlight_edge(rt2mod, tmp_path):
    d = tmp_path / "l"
    write(d, "m.mtl", "newmtl A\nKd 0.5 0.5 0.5\nKe 0 0 0\nnewmtl B\nKe 2 1 0\nnewmtl C\nKd 0.2 0.3 0.4\n"
                      "GlassHighlight\nnewmtl D\nEDGE_HIGHLIGHT\n")
    write(d, "m.obj", "mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl B\nf 1 2 3\n")
    m = load(rt2mod, d).materials()
    A, B, C_, D = m[1], m[2], m[3], m[4]
    assert A["materialType"] == rt2mod.DIFFUSE and A["emissionStrength"] == 0
    f = np.float32
    assert B["materialType"] == rt2mod.LIGHT
    assert B["emissionStrength"] == f(f(f(0.299) * f(2)) + f(f(0.587) * f(1))) + f(f(0.114) * f(0))
    assert C_["materialType"] == rt2mod.GLASS_HIGHLIGHT and np.allclose(C_["color"][:3], [0.2, 0.3, 0.4])
    assert D["isEdgeHighlight"] == 1


def test_textures_index_by_directory_order(rt2mod, tmp_path):
    d = tmp_path / "t"
    os.makedirs(d / "textures")
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "images")
    for n, src in (("b.png", "rgb8.png"), ("a.png", "gray8.png")):
        with open(os.path.join(golden, src), "rb") as f, open(d / "textures" / n, "wb") as g:
            g.write(f.read())
    write(d, "m.mtl", "newmtl T\nmap_Kd a.png\nnewmtl L\nKe 1 1 1\nmap_Kd b.png\n")
    write(d, "m.obj", "mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl T\nf 1 2 3\n")
    sd = load(rt2mod, d)
    names = [n for n in os.listdir(d / "textures")]
    assert sd.texture_names == names
    m = sd.materials()
    assert list(m["index"]) == [0, 2, 1]  # map order: L before T
    T, L = m[2], m[1]
    assert T["materialType"] == rt2mod.TEXTURE and T["textureIndex"] == names.index("a.png")
    assert L["materialType"] == rt2mod.LIGHT and L["textureIndex"] == -1  # lights ignore map_Kd
    # decoded and flipped on load, like Texture2D(path)
    assert sd.texture(names.index("a.png")).shape == (7, 13, 1)
    assert np.array_equal(sd.texture(names.index("b.png")),
                          rt2mod.load_image(os.path.join(golden, "rgb8.png"), flip_vertically=True))


def test_undecodable_texture_is_an_error(rt2mod, tmp_path):
    # Texture2D(path) throws when stbi_load fails (textureClass.cpp:96-101)
    d = tmp_path / "u"
    os.makedirs(d / "textures")
    (d / "textures" / "x.png").write_bytes(b"")
    write(d, "m.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    with pytest.raises(rt2mod.RT2Error, match="x.png"):
        load(rt2mod, d)


@pytest.mark.parametrize("files,err", [
    ({"m.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nf 1 2 3 4\n"}, "non-triangle"),
    ({"m.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3 \n"}, "non-triangle"),
    ({"m.obj": "mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl Nope\nf 1 2 3\n", "m.mtl": "newmtl A\n"},
     "not found"),
    ({"m.obj": "v 0 0 0\nf 1 2 3\n"}, "out of range"),
    ({"m.obj": "v 0 0 0\n", "README": "x"}, "extension"),
    ({"m.mtl": "newmtl A\nmap_Kd missing.png\n", "m.obj": "v 0 0 0\n"}, "texture not found"),
    ({"m.txt": "nothing"}, "OBJ file not found"),
])
def test_loader_errors(rt2mod, tmp_path, files, err):
    d = tmp_path / "e"
    for n, text in files.items():
        write(d, n, text)
    with pytest.raises(rt2mod.RT2Error, match=err):
        load(rt2mod, d)


def test_png_writer_roundtrip(rt2mod, tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (13, 17, 3), dtype=np.uint8)
    p = str(tmp_path / "x.png")
    rt2mod.write_png(p, img)
    raw = open(p, "rb").read()
    assert raw[:8] == b"\x89PNG\r\n\x1a\n"
    off, idat, ihdr = 8, b"", None
    while off < len(raw):
        n = struct.unpack(">I", raw[off:off + 4])[0]
        typ = raw[off + 4:off + 8]
        body = raw[off + 8:off + 8 + n]
        assert struct.unpack(">I", raw[off + 8 + n:off + 12 + n])[0] == zlib.crc32(typ + body)
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        if typ == b"IDAT":
            idat += body
        off += 12 + n
    assert ihdr[:4] == (17, 13, 8, 2)
    rows = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(13, 1 + 17 * 3)
    assert np.all(rows[:, 0] == 0)
    assert np.array_equal(rows[:, 1:].reshape(13, 17, 3), img)


def test_torus_generator_winding(rt2mod, tmp_path):
    from rt2 import generate_torus_obj
    folder = tmp_path / "torus"
    generate_torus_obj(str(folder), 20, 12)
    sd = load(rt2mod, folder)
    t = sd.triangles()
    assert len(t) == 2 * 20 * 12
    a, b, c = t["a"][:, :3].astype(np.float64), t["b"][:, :3].astype(np.float64), t["c"][:, :3].astype(np.float64)
    n = np.cross(b - a, c - a)
    cen = (a + b + c) / 3 - np.array([0, 2, 0])
    radial = cen.copy()
    radial[:, 1] = 0
    ring = radial / np.linalg.norm(radial, axis=1, keepdims=True) * 2.0
    outward = cen - ring
    assert np.all((n * outward).sum(1) > 0)  # e0 x e1 points out of the tube
