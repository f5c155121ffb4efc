"""Texture decoding (§8f row 3): rt2_image_load against the reference's own
stb_image (compiled from /root/reference by `make -C oracle ref`; fixtures made
by tests/golden/make_texture_golden.py): same size, channel count and pixel
bytes (sha256) after the vertical flip Texture2D requests."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "images.json")))
REF_DATA = "/root/reference/RayTracing/Data"

# stb_image decodes these; the product decoder rejects them by design
UNSUPPORTED = {"progressive.jpg": "progressive"}


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(GOLD["synthetic"]))
def test_synthetic_images_match_reference_stb(rt2mod, name):
    want = GOLD["synthetic"][name]
    path = os.path.join(HERE, "golden", "images", name)
    if name in UNSUPPORTED:
        with pytest.raises(rt2mod.RT2Error, match=UNSUPPORTED[name]):
            rt2mod.load_image(path)
        return
    img = rt2mod.load_image(path)
    assert img.shape == (want["height"], want["width"], want["channels"])
    assert digest(img) == want["sha256"], name


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference tree not mounted")
@pytest.mark.parametrize("rel", sorted(GOLD["reference"]))
def test_reference_textures_match_reference_stb(rt2mod, rel):
    want = GOLD["reference"][rel]
    img = rt2mod.load_image(os.path.join(REF_DATA, rel))
    assert img.shape == (want["height"], want["width"], want["channels"])
    assert digest(img) == want["sha256"], rel


def test_flip_and_errors(rt2mod, tmp_path):
    path = os.path.join(HERE, "golden", "images", "rgb8.png")
    a = rt2mod.load_image(path, flip_vertically=True)
    b = rt2mod.load_image(path, flip_vertically=False)
    assert np.array_equal(a, b[::-1])
    bad = tmp_path / "x.png"
    bad.write_bytes(b"\x89PNG\r\n\x1a\nnot really")
    with pytest.raises(rt2mod.RT2Error, match="x.png"):
        rt2mod.load_image(str(bad))
    junk = tmp_path / "y.bin"
    junk.write_bytes(b"hello")
    with pytest.raises(rt2mod.RT2Error, match="unknown image type"):
        rt2mod.load_image(str(junk))
    with pytest.raises(rt2mod.RT2Error, match="cannot open"):
        rt2mod.load_image(str(tmp_path / "missing.png"))


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference tree not mounted")
def test_loader_decodes_folder_textures(rt2mod):
    """getTrianglesData_ on a textured model: textures/ in directory order,
    decoded and flipped; TEXTURE materials index them (mesh.h:305-318, 430-450)."""
    sd = rt2mod.SceneData()
    sd.load_obj_folder(os.path.join(REF_DATA, "rin"))
    names = sd.texture_names
    assert sorted(names) == sorted(os.listdir(os.path.join(REF_DATA, "rin", "textures")))
    for i, n in enumerate(names):
        want = GOLD["reference"][f"rin/textures/{n}"]
        assert digest(sd.texture(i)) == want["sha256"]
    mats = sd.materials()
    tex = mats[mats["materialType"] == 5]
    assert len(tex) > 0 and (tex["textureIndex"] >= 0).all() and (tex["textureIndex"] < len(names)).all()
