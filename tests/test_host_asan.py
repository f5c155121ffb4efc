"""Host code under AddressSanitizer + UBSan (CPU only): the image decoders on
every golden image and 15k corrupted variants, the OBJ/MTL loader and BVH
build on 3k corrupted folders — each input decodes/loads or is rejected with
an error, with no invalid memory access or undefined behaviour
(tests/host_asan/fuzz_host.cpp)."""
import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_code_under_asan_and_ubsan():
    d = os.path.join(HERE, "host_asan")
    subprocess.run(["make", "-C", d], check=True, stdout=subprocess.DEVNULL, timeout=600)
    images = sorted(glob.glob(os.path.join(HERE, "golden", "images", "*")))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(d, "fuzz_host")] + images, capture_output=True, text=True, timeout=900,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "fuzzed 15200 corrupted images" in r.stdout
    assert "fuzzed 3000 corrupted OBJ/MTL folders" in r.stdout
