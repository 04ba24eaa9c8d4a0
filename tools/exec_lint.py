"""Lint for the round-2 overflow-kernel miscompile: a spill
or live-range copy of a VGPR into an AGPR (v_accvgpr_write) or to scratch,
placed in a basic block BEFORE that block's `s_or_b64 exec, exec, s[..]` --
i.e. in a control-flow join ("Flow") block while EXEC still holds the
divergent region's mask (empty after a divergent loop exits).  The copy then
writes only the region's lanes; a lane outside it later reads a stale value.
Only copies of a value that is live into the region (not written between
the region's s_and_saveexec and the copy) are reported: those are needed by
every lane; for an AGPR copy, only one read back after the restore (not a
save / restore pair inside the region).  (A heuristic over the text:
straight-line distance, no CFG.)

    python tools/exec_lint.py file.s ...            (hipcc --save-temps output)
    python tools/exec_lint.py --lib libhmpc.so      (disassembles the gfx950 code objects)

Prints every finding as kernel, line, instruction; exit status 1 if any."""
import os
import re
import subprocess
import sys
import tempfile

OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
SPILL = re.compile(r'^\s*(v_accvgpr_write_b32|scratch_store_\w+|buffer_store_\w+)\b')
RESTORE = re.compile(r'^\s*s_or_b64\s+exec,\s*exec,\s*s\[')
LABEL = re.compile(r'^(\.LBB\w+|[A-Za-z_][\w.$]*):')
KERNEL = re.compile(r'^([A-Za-z_][\w.$]*):\s*(;.*)?$')


VREG = re.compile(r'\bv(\d+)\b|\bv\[(\d+):(\d+)\]')
SAVEEXEC = re.compile(r'^\s*s_and_saveexec_b64\s+(s\[\d+:\d+\])')
NODEF = ('s_', 'ds_write', 'ds_store', 'global_store', 'scratch_store', 'buffer_store', 'flat_store',
         'v_cmp', 'v_readlane', 'v_readfirstlane', 'v_accvgpr_write', 'global_atomic', 'ds_add', 'ds_bpermute_no')


def _regs(tok):
    out = set()
    for m in VREG.finditer(tok):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _defs(ins):
    """VGPRs an instruction writes (its first operand), or an empty set."""
    op = ins.strip().split(None, 1)
    if len(op) < 2 or op[0].startswith(NODEF):
        return set()
    return _regs(op[1].split(',')[0])


def _live_in(prog, i_copy, mask, src):
    """Is `src` (a VGPR set) live into the divergent region that ends at the
    copy: not written between the region's s_and_saveexec (saving `mask`)
    and the copy?  Then every lane needs the value, not only the region's."""
    j = i_copy - 1
    while j >= 0:
        ins = prog[j][1]
        m = SAVEEXEC.match(ins)
        if m and m.group(1) == mask:
            return True
        if _defs(ins) & src:
            return False
        j -= 1
    return False


AREG = re.compile(r'\ba(\d+)\b')
AREAD = re.compile(r'^\s*v_accvgpr_read_b32\s+v\d+,\s*a(\d+)\b')
AWRITE = re.compile(r'^\s*v_accvgpr_write_b32\s+a(\d+)\b')


def _agpr_escapes(lines, k_copy, k_restore, areg):
    """An AGPR copy is a hazard only if its value is used OUTSIDE the region:
    not read back before the exec restore (a save / restore pair inside the
    region is region-local), and read after the restore before it is
    written again (straight-line scan to the kernel's end)."""
    for _, ins in lines[k_copy + 1:k_restore]:
        m = AREAD.match(ins)
        if m and int(m.group(1)) == areg:
            return False
    for _, ins in lines[k_restore + 1:]:
        if KERNEL.match(ins) and not ins.startswith('.LBB'):
            return False
        m = AREAD.match(ins)
        if m and int(m.group(1)) == areg:
            return True
        m = AWRITE.match(ins)
        if m and int(m.group(1)) == areg:
            return False
    return False


def lint_lines(lines, where, precise=True):
    out = []
    kernel, block = '?', []
    prog = []   # (line, instruction) of the current kernel, in order
    flat = [(ln, raw.split(';')[0].rstrip()) for ln, raw in lines]
    pos = {ln: k for k, (ln, _) in enumerate(flat)}
    for ln, raw in lines:
        line = raw.split(';')[0].rstrip() if not raw.lstrip().startswith(';') else ''
        m = LABEL.match(raw)
        if m:
            if KERNEL.match(raw) and not raw.startswith('.LBB'):
                kernel = m.group(1)
                prog = []
            block = []
            continue
        if not line.strip():
            continue
        mr = RESTORE.match(line)
        if mr:
            mask = line.split(',')[-1].strip()
            for bl, bi, bidx in block:
                if SPILL.match(bi):
                    ops = bi.strip().split(None, 1)[1]
                    src = _regs(ops.split(',')[1] if ops.startswith(('a', 'off')) or 'accvgpr' in bi else ops)
                    if precise and not _live_in(prog, bidx, mask, src):
                        continue
                    ma = AWRITE.match(bi)
                    if precise and ma and not _agpr_escapes(flat, pos[bl], pos[ln], int(ma.group(1))):
                        continue
                    out.append((where, kernel, bl, bi.strip()))
            block = []   # (later instructions run with the restored mask)
            prog.append((ln, line))
            continue
        prog.append((ln, line))
        if line.strip().startswith(('s_cbranch', 's_branch', 's_endpgm', 's_setpc')):
            block = []
            continue
        block.append((ln, line, len(prog) - 1))
    return out


def disasm_lib(path):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
    from test_kernel_resources import _code_objects
    res = []
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(_code_objects(path)):
            f = os.path.join(d, f'co{k}.o')
            open(f, 'wb').write(co)
            txt = subprocess.run([OBJDUMP, '-d', '--no-show-raw-insn', f], capture_output=True, text=True,
                                 check=True).stdout
            # objdump: "<symbol>:" headers and no .LBB labels; every branch
            # target starts a block, so treat any line ending a block as above
            lines = []
            for i, raw in enumerate(txt.splitlines()):
                m = re.match(r'^[0-9a-f]+ <(.+)>:', raw)
                if m:
                    lines.append((i, f'{m.group(1)}:'))
                    continue
                lines.append((i, raw.split('//')[0]))
            res += lint_lines(lines, f'{os.path.basename(path)}#co{k}')
    return res


def main():
    args = sys.argv[1:]
    found = []
    if args and args[0] == '--lib':
        for p in args[1:]:
            found += disasm_lib(p)
    else:
        for p in args:
            found += lint_lines(list(enumerate(open(p).read().splitlines(), 1)), p)
    for where, kern, ln, ins in found:
        print(f'{where}: {kern}: line {ln}: {ins}  (before the exec restore of its block)')
    print(f'{len(found)} finding(s)')
    return 1 if found else 0


if __name__ == '__main__':
    sys.exit(main())
