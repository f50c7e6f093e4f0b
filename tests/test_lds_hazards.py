"""Static check of the in-tree gfx950 kernels (tools/lds_hazards.py): no instruction touches a
register that an inline-asm ds_read still in flight will write.  The trunk kernels' fragment reads
are inline asm the compiler treats as complete when issued, so the register allocator may reuse a
register whose LDS load has not landed; the loops end with waits that name every fragment register
(the drains in csrc/conv_v7.hip).  Runs on the objects the in-tree build left (no GPU needed)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "alphazero-multi-game_amd", "build")
OBJS = ["conv_v7.o", "conv_bf16.o", "smallnet.o", "net_kernels.o", "tree_kernels.o", "engine.o"]


@pytest.mark.parametrize("obj", OBJS)
def test_no_inflight_lds_register_reuse(obj):
    path = os.path.join(BUILD, obj)
    if not os.path.exists(path):
        pytest.skip(f"{obj} not built (run __graft_entry__.build())")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lds_hazards.py"), path],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "kernels, 0 with hazards" in r.stdout
