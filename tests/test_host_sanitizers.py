"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the C ABI ("race
detection / sanitizers"): the library is rebuilt with -fsanitize=address,undefined on the HOST
compilation only (build.SAN_FLAGS, every flag behind -Xarch_host; device code unchanged, no GPU
sanitizer), and tests/host_abi_calls.py drives every entry point's validation and size arithmetic
in a child process with the shared ASan runtime preloaded. Any ASan report or UBSan runtime error
(e.g. a signed overflow in a range check) fails the test."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def test_c_abi_host_code_under_asan_ubsan():
    from deepinteract_amd import build
    lib = build.build_host_sanitized()
    env = dict(os.environ)
    env["LD_PRELOAD"] = build.asan_runtime()
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"           # CPython's arenas are not leaks
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([sys.executable, os.path.join(HERE, "host_abi_calls.py"), lib], env=env,
                       capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "host ABI calls:" in r.stdout and " ok" in r.stdout, out[-2000:]
