import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracing2-fork_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"

for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path)")
    config.addinivalue_line("markers", "reference: needs the reference tree at /root/reference")


def _ensure_built():
    lib = os.path.join(PKG, "rt2", "librt2.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)
    olib = os.path.join(ORACLE, "liboracle.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-C", ORACLE, "liboracle.so"], check=True, stdout=subprocess.DEVNULL)


_ensure_built()


def has_reference() -> bool:
    return os.path.isdir(os.path.join(REFERENCE, "RayTracing", "Data"))


needs_reference = pytest.mark.skipif(not has_reference(), reason="reference tree not mounted (GPU box)")


@pytest.fixture(scope="session")
def rt2mod():
    import rt2
    rt2.lib()
    return rt2


@pytest.fixture(scope="session")
def oraclemod():
    import oracle
    oracle.lib()
    return oracle


_scene_cache = {}


@pytest.fixture(scope="session")
def config_scene(rt2mod, tmp_path_factory):
    def get(name):
        if name not in _scene_cache:
            _scene_cache[name] = rt2mod.build_config_scene(name, str(tmp_path_factory.mktemp("scenes")))
        return _scene_cache[name]
    return get


# The experiment build (make EXPERIMENTS=1, RT2_LIB=exp) adds the A/B kernel
# variants; their parity tests are collected only when it is loaded.
EXPERIMENTS = os.environ.get("RT2_LIB") == "exp"
collect_ignore = [] if EXPERIMENTS else ["test_gpu_experiments.py"]


def require_variant(rt2mod, v):
    """Skips the calling test when kernel variant v is not in the loaded build
    (A/B experiment variants: make EXPERIMENTS=1, RT2_LIB=exp)."""
    if not rt2mod.has_variant(v):
        # the experiment build carries every listed variant: one missing there
        # is a lost kernel, not a skip
        if EXPERIMENTS:
            pytest.fail(f"variant {v} is listed but missing from the experiment build")
        pytest.skip(f"variant {v} is an experiment variant (not in the product build)")
