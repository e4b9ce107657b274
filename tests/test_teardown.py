"""Handle teardown order (round-2 exit-time SIGSEGV): every C handle still alive at interpreter
exit is destroyed by ompl_amd.abi's atexit hook, newest first, and no destroy call runs after
that hook (so none reaches a HIP runtime the C library's static teardown has already shut
down).  CPU-only: the handles here record their destroy calls instead of calling the library."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import ctypes as C, sys
sys.path.insert(0, %r)
from ompl_amd import abi

class Rec(abi.Handle):
    def __init__(self, name):
        self.name = name
        self._own(C.c_void_p(0x1000 + len(name)))
    def _destroy(self, h):
        print("destroy", self.name, flush=True)

a, b, c = Rec("a"), Rec("bb"), Rec("ccc")
d = Rec("dddd"); d.close(); d.close()   # explicit close: once, idempotent
with Rec("eeeee") as e:
    pass
cyc = Rec("ffffff"); cyc.self_ref = cyc   # a cycle the GC would collect only at finalisation
del cyc
print("exit", flush=True)
'''


def test_atexit_closes_newest_first_and_nothing_after():
    out = subprocess.run([sys.executable, "-c", SCRIPT % ROOT], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, OMPL_GPU_NO_TORCH="1"))
    assert out.returncode == 0, out.stderr
    lines = out.stdout.split("\n")
    lines = [l for l in lines if l]
    assert lines[:2] == ["destroy dddd", "destroy eeeee"]
    assert lines[2] == "exit"
    # the atexit hook: newest first (the cycle member is still alive), then nothing more
    assert lines[3:] == ["destroy ffffff", "destroy ccc", "destroy bb", "destroy a"]


def test_closed_handle_is_not_destroyed_twice():
    from ompl_amd import abi
    calls = []

    class Rec(abi.Handle):
        def _destroy(self, h):
            calls.append(h.value)

    import ctypes as C
    r = Rec()
    r._own(C.c_void_p(0x1234))
    r.close()
    r.close()
    del r
    assert calls == [0x1234]
