"""Debug build and sanitizer subsystem.

* host code under AddressSanitizer + UBSan (tools/sanitize/run_host_asan.sh), with a canary that must be caught;
* the DTF_DEBUG device-check macros compile for gfx950;
* the debug-library launch wrapper (ops._DebugLib) on fakes (CPU) and on the real debug build (GPU).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
needs_hipcc = pytest.mark.skipif(not os.path.isfile(HIPCC), reason="hipcc not installed")


@needs_hipcc
def test_host_code_under_asan_ubsan(tmp_path):
    script = os.path.join(ROOT, "tools", "sanitize", "run_host_asan.sh")
    if not os.path.isfile(script):
        pytest.skip("tools/sanitize not shipped to this machine (.gpurunignore: host-only CPU check)")
    ok = subprocess.run(["bash", script, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stdout + ok.stderr
    assert "host_check: ok" in ok.stdout
    bad = subprocess.run([str(tmp_path / "host_check"), "--canary"], capture_output=True, text=True, timeout=60)
    assert bad.returncode != 0 and "heap-buffer-overflow" in bad.stderr, bad.stdout + bad.stderr


@needs_hipcc
def test_debug_macros_compile_for_gfx950(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text('#include "common.h"\n'
                   "__global__ void k(const int* w, int* o) { DTF_WG_CHECK(w[blockIdx.x] > 0); o[blockIdx.x] = 1; }\n"
                   "DTF_DEBUG_EXPORT(k)\n"
                   "DTF_API int launch_k(const int* w, int* o, int n) {\n"
                   "  DTF_HOST_CHECK(n > 0 && DTF_ALIGNED16(w));\n"
                   "  hipLaunchKernelGGL(k, dim3(n), dim3(64), 0, 0, w, o); return DTF_CHECK_LAUNCH(); }\n")
    inc = os.path.join(ROOT, "distributedtf_amd", "ops", "csrc")
    for extra in ([], ["-DDTF_DEBUG=1"]):
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-I", inc, "-c", str(src), "-o",
                            str(tmp_path / "k.o")] + extra, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr


def test_debug_lib_wrapper_checks(monkeypatch):
    import torch
    from distributedtf_amd import ops

    class FakeFn:
        def __init__(self, rc):
            self.rc, self.calls, self.argtypes = rc, 0, None

        def __call__(self, *a):
            self.calls += 1
            return self.rc

    class FakeLib:
        dtf_good = FakeFn(0)
        dtf_hostbad = FakeFn(100000 + 42)
        dtf_args_size = FakeFn(7)
        dtf_debug_error_conv = FakeFn(0)

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(ops._build, "CSRC", os.path.join(ROOT, "distributedtf_amd", "ops", "csrc"))
    L = ops._DebugLib(FakeLib())
    assert L.dtf_good() == 0 and L.launches == 1
    L.dtf_good.argtypes = ["x"]  # forwarded to the underlying function
    assert FakeLib.dtf_good.argtypes == ["x"]
    assert L.dtf_args_size() == 7 and L.launches == 1  # ABI probes are not launches
    with pytest.raises(RuntimeError, match="host-side argument check failed .csrc line 42"):
        L.dtf_hostbad()
    FakeLib.dtf_debug_error_conv.rc = 1234
    with pytest.raises(RuntimeError, match="device check failed in conv.hip line 1234"):
        L.dtf_good()


@pytest.mark.gpu
def test_debug_build_on_gpu():
    from distributedtf_amd.ops import build as kb
    if not os.path.isfile(kb.LIB_DEBUG):
        pytest.fail("debug kernel library missing: run __graft_entry__.build()")
    env = dict(os.environ, DTF_DEBUG="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "_debug_probe.py")], env=env,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "debug probe ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--model", "mnist", "--pop", "2", "--batch", "16"],
                                  ["--model", "imagenet", "--pop", "2", "--batch", "2"]])
def test_debug_build_other_families_on_gpu(args):
    """MNIST and ImageNet steps through the debug library: every launch synchronised and checked."""
    env = dict(os.environ, DTF_DEBUG="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
                        "--exploit_every", "0"] + args, env=env, capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert '"metric"' in r.stdout
