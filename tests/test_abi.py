"""The C-ABI library loads and exports every symbol include/rl_hip.h declares (CPU only:
no compute calls). Struct layouts in the Python binding match the C header."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

import hiprl

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rl_hip.h"


def declared_functions():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(rl_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_all_declared_symbols():
    lib = hiprl.load_library()
    names = declared_functions()
    assert len(names) >= 14
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(n for n, _, _ in hiprl.ABI) == names
    assert lib.rl_abi_version() == hiprl.ABI_VERSION == 7


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include "rl_hip.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(){printf('
                   '"%zu %zu %zu %zu %zu %zu %zu %zu %zu %d %d %zu %zu %zu\\n",'
                   'sizeof(rl_config),sizeof(rl_rule),sizeof(rl_batch),sizeof(rl_status),sizeof(rl_engine_stats),'
                   'offsetof(rl_config,hash_seed),offsetof(rl_config,max_load_permille),sizeof(rl_occupancy),'
                   'sizeof(rl_host_batch),RL_BLOB_SLACK,RL_MAX_IN_FLIGHT,sizeof(rl_router_config),sizeof(rl_router_stats),'
                   'offsetof(rl_router_stats,pack_us));printf("%zu %zu %zu %zu %zu\\n",sizeof(rl_batch_c),'
                   'offsetof(rl_batch_c,now_base),offsetof(rl_batch_c,req_of),sizeof(rl_host_batch_c),'
                   'sizeof(struct rl_raw_reply));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [C.sizeof(hiprl.RlConfig), C.sizeof(hiprl.RlRule), C.sizeof(hiprl.RlBatch), hiprl.STATUS_DTYPE.itemsize,
            C.sizeof(hiprl.RlEngineStats), hiprl.RlConfig.hash_seed.offset, hiprl.RlConfig.max_load_permille.offset,
            C.sizeof(hiprl.RlOccupancy), C.sizeof(hiprl.RlHostBatch), hiprl.BLOB_SLACK, hiprl.MAX_IN_FLIGHT, C.sizeof(hiprl.RlRouterConfig),
            C.sizeof(hiprl.RlRouterStats), hiprl.RlRouterStats.pack_us.offset,
            C.sizeof(hiprl.RlBatchC), hiprl.RlBatchC.now_base.offset, hiprl.RlBatchC.req_of.offset,
            C.sizeof(hiprl.RlHostBatchC), hiprl.RAW_DTYPE.itemsize]
    assert got == want
    assert hiprl.STATUS_DTYPE.itemsize == 20


def test_null_and_bad_arguments_do_not_touch_the_gpu():
    lib = hiprl.load_library()
    out = C.c_void_p()
    assert lib.rl_create(None, C.byref(out)) == -1
    cfg = hiprl.RlConfig()
    cfg.struct_size = 3  # wrong ABI size
    assert lib.rl_create(C.byref(cfg), C.byref(out)) == -1
    assert lib.rl_wait(None) == -1
    # with no engine: the calling thread's last rl_create failure (none has touched HIP here)
    assert lib.rl_last_error(None) == b"no rl_create failure on this thread"
