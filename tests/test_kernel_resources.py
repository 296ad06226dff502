"""Register and scratch budgets of the benched kernels, read from the built
library's gfx950 code objects (AMDGPU metadata notes; CPU only).

The launch shapes depend on them:
  * step_kernel<7, 1> (the headline) holds 4 one-wave envs per SIMD, so all
    4096 envs are resident at once on 1024 SIMDs: <= 128 VGPRs;
  * wg_step_kernel<7> (config 4) fits 4 workgroups of 4 waves per CU at
    <= 128 registers (with its <= 40 KiB of LDS): config 4's 1024-env share
    of a GPU is resident in ONE dispatch round on 256 CUs.  At 159
    registers (round 5) 3 fit and the last 256 envs ran as a second round;
    the fixed LDS layout and the per-step opaque thread index (gw_rtt.inc
    wg_carve / wg_fresh) took it to 123;
  * the workgroup and headline kernels touch no scratch: every scratch-using
    build of the workgroup kernel measured slower (profiles/r04/ab_wg_min_waves.txt);
  * pac_kernel runs 6 waves per SIMD (config 5: 16384 envs).
"""
import os
import re
import struct

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'abmarl_amd', '_build', 'libgw_engine.so')


def _sections(d):
    shoff = struct.unpack_from('<Q', d, 0x28)[0]
    ent, num, stri = struct.unpack_from('<HHH', d, 0x3A)
    secs = [struct.unpack_from('<IIQQQQIIQQ', d, shoff + i * ent) for i in range(num)]
    so = secs[stri][4]
    return {d[so + s[0]:d.index(b'\0', so + s[0])].decode(): s for s in secs}


def code_objects(path=LIB):
    """The gfx950 code objects (ELF images) in the library's offload bundles
    (.hip_fatbin)."""
    data = open(path, 'rb').read()
    fb = _sections(data)['.hip_fatbin']
    blob = data[fb[4]:fb[4] + fb[5]]
    out = []
    for st in [m.start() for m in re.finditer(b'__CLANG_OFFLOAD_BUNDLE__', blob)]:
        n = struct.unpack_from('<Q', blob, st + 24)[0]
        p = st + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if 'gfx950' in triple:
                out.append(blob[st + off:st + off + size])
    return out


def kernel_metadata(path=LIB):
    """{kernel symbol: metadata map} of every gfx950 code object in the
    library's offload bundles (.hip_fatbin)."""
    import msgpack
    out = {}
    for co in code_objects(path):
        ns = _sections(co)['.note']
        note, q = co[ns[4]:ns[4] + ns[5]], 0
        while q < len(note):
            nsz, dsz, typ = struct.unpack_from('<III', note, q)
            q += 12
            name = note[q:q + nsz]
            q += (nsz + 3) & ~3
            desc = note[q:q + dsz]
            q += (dsz + 3) & ~3
            if name.startswith(b'AMDGPU') and typ == 32:
                for k in msgpack.unpackb(desc, raw=False)['amdhsa.kernels']:
                    out[k['.name']] = k
    return out


@pytest.fixture(scope='module')
def md():
    if not os.path.exists(LIB):
        pytest.skip('engine library not built')
    pytest.importorskip('msgpack')
    return kernel_metadata()


def _get(md, pattern):
    hits = [v for k, v in md.items() if re.search(pattern, k)]
    assert len(hits) == 1, (pattern, len(hits))
    return hits[0]


def _granules(v):
    return (v + 7) // 8 * 8


def test_headline_kernel_four_envs_per_simd(md):
    k = _get(md, r'11step_kernelILi7ELi1E')
    assert _granules(k['.vgpr_count']) <= 128, k['.vgpr_count']
    assert k['.private_segment_fixed_size'] == 0


def test_workgroup_kernel_four_per_cu(md):
    k = _get(md, r'14wg_step_kernelILi7E')
    assert _granules(k['.vgpr_count']) <= 512 // 4, k['.vgpr_count']
    assert k['.private_segment_fixed_size'] == 0
    # static LDS + config 4's dynamic LDS (gw_rtt.inc wg_smem_bytes: 64x64,
    # 256 lanes, S = 7, 3 encodings, 4 waves) within a quarter of 160 KiB
    assert k['.group_segment_fixed_size'] + config4_lds_bytes() <= 160 * 1024 // 4


def _a16(n):
    return (n + 15) // 16 * 16


def config4_lds_bytes(H=64, W=64, A=256, S=7, max_enc=3, nwv=4, max_lanes=256, wave=64, mt_n=624):
    """wg_smem_bytes of gw_rtt.inc for config 4 (the fixed per-lane part,
    the work union, the padded cell table, counts and blocker bitmap)."""
    m_words = 64 + 3 * 64
    lut = S * S * ((S * S + 31) // 32)
    fixed = 6 * 4 * max_lanes + 2 * 8 * max_lanes + 4 * wave * 4 + 4 * m_words + 4 * mt_n
    fixed = _a16(fixed + 4 * (lut if lut <= 256 else 0))
    HW = H * W
    cnt = _a16((HW + 3) // 4 * 4)
    st = _a16(A * S * ((S + 3) & ~3))
    st = max(st, 2 * cnt, _a16((max_enc + 1) * 64 * 8) + _a16(A * 4),
             4 * 640 + 4 * mt_n + 4 * wave * nwv + 8 * (15 + 1) * 4) + 16
    pad = S // 2                  # config 4: the target's attack range <= its view range
    pitch = (W + 2 * pad + 3) // 4 * 4 + 4 * ((S + 3) // 4 + 1)
    tbl = _a16((H + 2 * pad + 1) * pitch)
    return fixed + st + tbl + cnt + _a16(((HW + 31) // 32 + 2) * 4)


def test_pacman_kernel_six_per_simd(md):
    """pac_kernel's step protocols at 6 waves per SIMD (launch bound; up to 32 B
    of spill measured faster than 5 waves without, profiles/r04/ab_pac_waves*)."""
    for pattern in (r'10pac_kernelILi3E', r'10pac_kernelILi4E'):
        k = _get(md, pattern)
        assert _granules(k['.vgpr_count']) <= 512 // 6, k['.vgpr_count']
        assert k['.private_segment_fixed_size'] <= 32


def test_maze_kernel_without_scratch(md):
    assert _get(md, r'16lane_step_kernelILi5ELi10E')['.private_segment_fixed_size'] == 0


OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'


def twist_memory_ops(path):
    """{function: set of memory opcodes} of every MT19937 twist block in the
    library's gfx950 code: the 0x9908b0df mask of mt19937's twist and the 25
    instructions before it, where the key words are read."""
    import subprocess
    import tempfile
    found = {}
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix='.co') as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([OBJDUMP, '-d', '--mcpu=gfx950', f.name], check=True,
                                 capture_output=True, text=True).stdout.split('\n')
        fn = None
        for i, ln in enumerate(txt):
            m = re.match(r'^[0-9a-f]+ <(.+)>:', ln)
            if m:
                fn = m.group(1)
            elif '0x9908b0df' in ln:
                ops = {x.split()[0] for x in txt[max(0, i - 25):i]
                       if x.strip().startswith(('flat_', 'ds_', 'global_', 'scratch_', 'buffer_'))
                       for x in [x.strip()]}
                found.setdefault(fn, set()).update(ops)
    return found


def flat_functions(path):
    """({function: number of flat_* instructions}, {functions that form a
    generic LDS address: src_shared_base}) of the library's gfx950 code."""
    import subprocess
    import tempfile
    flat, shared = {}, set()
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix='.co') as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([OBJDUMP, '-d', '--mcpu=gfx950', f.name], check=True,
                                 capture_output=True, text=True).stdout.split('\n')
        fn = None
        for ln in txt:
            m = re.match(r'^[0-9a-f]+ <(.+)>:', ln)
            if m:
                fn = m.group(1)
            elif ln.strip().startswith('flat_'):
                flat[fn] = flat.get(fn, 0) + 1
            if 'src_shared_base' in ln:
                shared.add(fn)
    return flat, shared


def _lib(variant):
    from abmarl_amd import _native
    path = _native.variant_lib(variant)
    if not os.path.exists(path):
        pytest.skip(f'{os.path.basename(path)} not built')
    if not os.path.exists(OBJDUMP):
        pytest.skip('llvm-objdump missing')
    return path


@pytest.mark.parametrize('variant', ['', 'checks'])
def test_mt_key_never_read_through_flat(variant):
    """Every MT19937 twist in every kernel reads the key with ds_* operations:
    the key pointer is LDS-typed (lds_u32) everywhere.  The round-4 memory
    aperture violation: a generic key pointer, held in a scratch-resident Rng
    (the generic-window kernels), made the inlined twist flat_* accesses, and
    LLVM folded part of the key[i - 227] index into the instruction's
    immediate offset -- `flat_load_dword v, v[a:b] offset:768` with the VGPR
    address key + 4 * lane - 908, below the LDS aperture base (the key is at
    LDS offset 0), which selects no aperture (DESIGN §4 "MT19937 key
    addressing", tools/fault_r05/)."""
    ops = twist_memory_ops(_lib(variant))
    assert ops, 'no twist found in the library'
    bad = {fn: sorted(o) for fn, o in ops.items() if any(x.startswith('flat_') for x in o)}
    assert not bad, bad
    assert all(any(x.startswith('ds_') for x in o) for o in ops.values()), ops


@pytest.mark.parametrize('variant', ['', 'checks'])
def test_no_generic_lds_pointer(variant):
    """No kernel forms a generic (flat) address of LDS -- src_shared_base,
    the LDS aperture, appears nowhere -- so no flat_* instruction can reach
    LDS, and no folded immediate offset can push a flat LDS address out of
    its aperture (the round-4 fault, which 95ec8c4's reset_kernel<0> shows
    with its two src_shared_base materialisations of the key pointer).  The
    production step / reset / rollout kernels have no flat_* instruction at
    all; the component-API kernels and the checks build keep flat loads of
    the global arrays behind a Params copy in scratch."""
    flat, shared = flat_functions(_lib(variant))
    assert not shared, sorted(shared)
    if variant == '':
        bad = {fn: n for fn, n in flat.items() if 'comp_kernel' not in fn}
        assert not bad, bad
