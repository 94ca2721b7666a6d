"""The generated DPP step headers (tools/gen_dpp16.py -> ba_dpp16.h, ba_dpp16f.h) are what the
generator writes (no hand edits), and every asm block of the fused steps keeps the gfx950 wait
states the compiler cannot insert inside inline asm, checked here independently of the
generator's own bookkeeping: 2 between a VALU write of a VGPR and a DPP read of it (a block's
first DPP read assumes a write just before the block), 1 between a transcendental's result and
its first use."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "orb_slam3_ros2_amd", "csrc")


def test_headers_match_generator(tmp_path):
    env = dict(os.environ, ORBHIP_GEN_OUT=str(tmp_path))
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_dpp16.py")], env=env, check=True,
                   capture_output=True)
    for name in ("ba_dpp16.h", "ba_dpp16f.h"):
        with open(os.path.join(CSRC, name)) as a, open(tmp_path / name) as b:
            assert a.read() == b.read(), name


def _blocks(text):
    for m in re.finditer(r"asm(?: volatile)?\((.*?)\n\s*:", text, re.S):
        yield [x for x in re.findall(r'"([^"]*?)\\n\\t"', m.group(1))]


def _operands(ins):
    return re.findall(r"%\[(\w+)\]", ins)


def test_fused_blocks_wait_states():
    with open(os.path.join(CSRC, "ba_dpp16f.h")) as f:
        text = f.read()
    nblocks = 0
    for block in _blocks(text):
        nblocks += 1
        since = {}          # register -> wait states since its last write in the block
        start = 0           # wait states since the block began: a register not written in the block
        #                     counts from there (it may have been written just before the block)
        trans_dst = None    # destination of the previous instruction if it was a transcendental
        for ins in block:
            if ins.startswith("s_nop"):
                n = int(ins.split()[1]) + 1
                for r in since:
                    since[r] += n
                start += n
                trans_dst = None
                continue
            ops = _operands(ins)
            dst, srcs = ops[0], ops[1:]
            if "_dpp" in ins:
                src0 = srcs[0]
                assert since.get(src0, start) >= 2, (ins, since.get(src0, start), block)
            if trans_dst is not None:
                assert trans_dst not in srcs, (ins, "reads a transcendental result with no wait state")
            for r in since:
                since[r] += 1
            start += 1
            since[dst] = 0
            trans_dst = dst if ins.startswith("v_rcp") or ins.startswith("v_rsq") else None
    assert nblocks == 16
