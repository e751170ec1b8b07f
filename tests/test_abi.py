"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/kubecheck.h declares, and fails loudly (negative errno + a
message, no abort) when no GPU is present."""
import ctypes as C
import os
import re
import subprocess

import pytest

import kubecheck
from kubecheck import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kubecheck.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kc_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_exported():
    syms = declared_symbols()
    assert len(syms) >= 40
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (kc_\w+)", out))
    assert not (set(syms) - exported), set(syms) - exported
    # and the ctypes table covers them all
    assert {s for s, _, _ in _lib.SIGNATURES} == set(syms)


def test_abi_version_and_info():
    lib = kubecheck.load()
    assert lib.kc_abi_version() == 1
    assert b"gfx950" in lib.kc_build_info()


def test_bad_arguments_return_einval():
    lib = kubecheck.load()
    assert lib.kc_engine_create(None, None) == -22
    assert b"NULL" in lib.kc_last_error()
    cfg = _lib.KcModelConfig()
    lib.kc_model_config_default(C.byref(cfg))
    assert (cfg.nc, cfg.np, cfg.ns, cfg.can_fail, cfg.can_timeout, cfg.check_deadlock) == (1, 1, 1, 1, 1, 1)
    cfg.nc = 7
    h = C.c_void_p()
    assert lib.kc_engine_create(C.byref(cfg), C.byref(h)) == -22
    assert b"unsupported model" in lib.kc_last_error()


@pytest.mark.skipif(kubecheck.device_count() > 0, reason="checks the no-GPU failure mode")
def test_no_gpu_fails_loudly():
    with pytest.raises(kubecheck.KubecheckError) as e:
        kubecheck.ModelChecker()
    assert e.value.code == -19 and "no CPU fallback" in str(e.value)
    with pytest.raises(kubecheck.KubecheckError):
        kubecheck.FPSet(1024)
    with pytest.raises(kubecheck.KubecheckError):
        kubecheck.StateQueue(4, 16)


def test_spec_words():
    assert kubecheck.Spec(kubecheck.ModelConfig()).state_words == 4        # 32 B per Model_1 state
    assert kubecheck.Spec(kubecheck.ModelConfig(np=2)).state_words == 6    # 48 B for NP=2
    assert kubecheck.Spec(kubecheck.ModelConfig()).tuple_words == 1 + 19 * 3


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of the C structs have the header's sizes and field
    offsets (compiled with the host C compiler against include/kubecheck.h)."""
    structs = {"kc_model_config": _lib.KcModelConfig, "kc_result": _lib.KcResult,
               "kc_squeue_config": _lib.KcSqueueConfig, "kc_squeue_stats": _lib.KcSqueueStats,
               "kc_host_comm": _lib.KcHostComm}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "kubecheck.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'  printf("{cname}.{f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for f in py._fields_:
            assert int(got[f"{cname}.{f[0]}"]) == getattr(py, f[0]).offset, (cname, f[0])


def test_model_config_carries_tlc_order():
    # ModelConfig.tlc_order (round 5: TLC-ordered claims at R > 1) reaches
    # the C struct; the default stays off
    from kubecheck import ModelConfig
    assert ModelConfig().to_c().tlc_order == 0
    assert ModelConfig(tlc_order=True).to_c().tlc_order == 1
    assert ModelConfig().to_c().first_claim == 0
    assert ModelConfig(first_claim=True).to_c().first_claim == 1
