"""Host-side AddressSanitizer run of the C-ABI layer (SURVEY.md §5 "Race detection / sanitizers"):
`make asan` builds dmip_capi.cpp with -fsanitize=address (host code only; GPU sanitizers are not
available on this pool), links it with the regular kernel objects, and tests/asan/capi_args.cpp drives
every entry point's argument validation and the thread-local error buffer. CPU only."""
import os
import subprocess

import pytest

from conftest import ROOT

OBJ = os.path.join(ROOT, "diffusion-modelling-for-inverse-problems_amd", "csrc", "dmip_kernels.o")


def test_capi_argument_validation_under_asan():
    if not os.path.exists(OBJ):
        pytest.skip("kernel objects not built (make)")
    r = subprocess.run(["make", "-C", ROOT, "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "capi_args")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "ok: 0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr
