"""Build the in-tree native libraries (no pip, no JIT cache).

  aero-cli_amd/libaero_engine.so   product: HIP kernels for gfx950 + C ABI
  tools/libaero_synth.so           synthetic Aero P-channel transmitter
  oracle/liboracle.so              test-only CPU restatement (checker)

Usage: python aero-cli_amd/build.py [--engine] [--synth] [--oracle] [-j N]
(no flag = everything).  Object files go to aero-cli_amd/build/.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, 'build')
ENGINE_SO = os.path.join(HERE, 'libaero_engine.so')
SYNTH_SO = os.path.join(ROOT, 'tools', 'libaero_synth.so')
ORACLE_DIR = os.path.join(ROOT, 'oracle')

ARCH = os.environ.get('AERO_OFFLOAD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', shutil.which('hipcc') or '/opt/rocm/bin/hipcc')
# bit-exactness: no FP contraction, no fast math, anywhere on the product path
FP = ['-ffp-contract=off', '-fno-fast-math']
HIP_FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH] + FP
CXX_FLAGS = ['-O2', '-std=c++17', '-fPIC', '-Wall'] + FP

HIP_SRCS = ['demod_oqpsk.hip', 'demod_msk.hip', 'coarse.hip', 'aerol.hip', 'engine.hip', 'chan.hip', 'burst.hip', 'burst_msk.hip',
            'burst_engine.hip', 'cchan.hip']
CXX_SRCS = ['tables_host.cpp', 'acars_host.cpp']
# Per-file codegen: the burst demodulators' loops hold their state in
# registers; LLVM's machine LICM hoists every FP64 constant of the inlined
# libm ports out of the loop into SGPRs, hundreds of them, which then spill
# (AGPR / VGPR-lane round trips every sample).  Without it they stay
# rematerialised at their use.
# The continuous OQPSK demod schedules better with memory clauses kept
# together (its loop's table gathers and ring loads issue back to back):
# 14.9 -> 14.6 ms per hop (profiles/r03/ab/round3c/ab_sched_*.log; max-ilp
# 14.8, and both strategies slow the coarse kernel, which keeps the default).
# With the RRC partial sums on the helper wave, machine LICM's hoisted FP64
# constants are what spills (211 SGPRs -> VGPR lanes; 15 without it):
# 13.76 -> 12.83 ms (profiles/r04/ab/g8_licm.txt).
FILE_FLAGS = {'burst.hip': ['-mllvm', '-disable-machine-licm'],
              'burst_msk.hip': ['-mllvm', '-disable-machine-licm'],
              'demod_oqpsk.hip': ['-mllvm', '--amdgpu-sched-strategy=max-memory-clause', '-mllvm',
                                  '-disable-machine-licm'],
              'cchan.hip': ['-mllvm', '-disable-machine-licm']}


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('build failed: %s\n%s%s' % (' '.join(cmd), r.stdout, r.stderr))
    return r


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_engine(jobs=4, variant=None, defines=(), file_flags=None):
    """Builds aero-cli_amd/libaero_engine.so.  `variant`/`defines`/`file_flags`
    build an experimental copy (libaero_engine_<variant>.so, objects in
    build/<variant>) for A/B kernel measurements; select it with
    AERO_ENGINE_SO=<path>."""
    ff = dict(FILE_FLAGS, **(file_flags or {}))
    bdir = BUILD if variant is None else os.path.join(BUILD, variant)
    out = ENGINE_SO if variant is None else os.path.join(HERE, 'libaero_engine_%s.so' % variant)
    os.makedirs(bdir, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith('.h')]
    headers += [os.path.join(ROOT, 'include', h) for h in ('aero_engine.h', 'aero_chan.h')]
    dflags = ['-D' + d for d in defines]
    tasks, objs = [], []
    for s in HIP_SRCS + CXX_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(bdir, s + '.o')
        objs.append(obj)
        if _stale(obj, [src] + headers):
            if s.endswith('.hip'):
                cmd = [HIPCC] + HIP_FLAGS + ff.get(s, []) + dflags + ['-c', src, '-o', obj]
            else:
                cmd = ['g++'] + CXX_FLAGS + dflags + ['-c', src, '-o', obj]
            tasks.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, t) for t in tasks]:
            f.result()
    if tasks or _stale(out, objs):
        _run([HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', out] + objs)
    return out


def build_synth():
    src = os.path.join(ROOT, 'tools', 'aero_synth.cpp')
    if _stale(SYNTH_SO, [src]):
        _run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-o', SYNTH_SO, src, '-lm'])
    return SYNTH_SO


MATHHOST_SO = os.path.join(ROOT, 'tools', 'libaero_mathhost.so')
FFTSIM_SO = os.path.join(ROOT, 'tools', 'libfft_chain_sim.so')


def build_fftsim():
    """Test-only host model of the coarse kernel's FFT layouts (tests/test_fft_chain_sim.py)."""
    src = os.path.join(ROOT, 'tools', 'fft_chain_sim.cpp')
    if _stale(FFTSIM_SO, [src, os.path.join(CSRC, 'fft_layout.h')]):
        _run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off', '-o', FFTSIM_SO, src])
    return FFTSIM_SO


def build_mathhost():
    src = os.path.join(ROOT, 'tools', 'mathhost.cpp')
    deps = [src, os.path.join(CSRC, 'aero_math.h'), os.path.join(CSRC, 'aero_glibc_tables.h')]
    if _stale(MATHHOST_SO, deps):
        _run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off', '-o', MATHHOST_SO, src, '-lm'])
    return MATHHOST_SO


HOSTCHECK_SO = os.path.join(ROOT, 'tools', 'libaero_hostcheck.so')
HOSTCHECK_SRCS = [os.path.join(ROOT, 'tools', 'hostcheck.cpp'), os.path.join(CSRC, 'acars_host.cpp'),
                  os.path.join(CSRC, 'tables_host.cpp')]


def build_hostcheck(out=HOSTCHECK_SO, extra=()):
    """Test-only CPU harness over the engine's host C++ (acars_host, tables_host)."""
    deps = HOSTCHECK_SRCS + [os.path.join(CSRC, h) for h in ('acars_host.h', 'tables_host.h')]
    if _stale(out, deps):
        _run(['g++'] + CXX_FLAGS + list(extra) + ['-shared', '-o', out] + HOSTCHECK_SRCS + ['-lm'])
    return out


def build_oracle():
    _run(['make', '-s', '-C', ORACLE_DIR])
    # the reference's own Qt-free sources (JFFT, Oscillator) as a second
    # checker, only where the reference tree exists (not on the GPU box)
    if os.path.isdir('/root/reference'):
        _run(['make', '-s', '-C', ORACLE_DIR, 'ref'])
    return os.path.join(ORACLE_DIR, 'liboracle.so')


HOST = os.path.join(HERE, 'host')
BIN = os.path.join(HERE, 'bin')
HOST_COMMON = ['qstr.cpp', 'output.cpp', 'forwarder.cpp', 'zmq_dl.cpp', 'ini.cpp']
# the host binaries: drop-in aero-decode / aero-publish over the engine's C ABI
HOST_BINS = {'aero-decode': ['aero_decode.cpp'], 'aero-publish': ['aero_publish.cpp']}
TOOL_BINS = {'zmq_pcm_pub': os.path.join(ROOT, 'tools', 'zmq_pcm_pub.cpp')}


def build_host(jobs=4):
    """aero-cli_amd/bin/<binary>: C++17 over include/aero_engine.h, linked
    to libaero_engine.so through an $ORIGIN rpath; libzmq is dlopen'ed."""
    os.makedirs(BIN, exist_ok=True)
    hdrs = [os.path.join(HOST, h) for h in os.listdir(HOST) if h.endswith('.h')]
    hdrs += [os.path.join(ROOT, 'include', 'aero_engine.h'), os.path.join(ROOT, 'include', 'aero_chan.h')]
    bdir = os.path.join(BUILD, 'host')
    os.makedirs(bdir, exist_ok=True)
    objs = {}
    tasks = []
    for s in HOST_COMMON + sum(HOST_BINS.values(), []):
        src, obj = os.path.join(HOST, s), os.path.join(bdir, s + '.o')
        objs[s] = obj
        if _stale(obj, [src] + hdrs):
            tasks.append(['g++', '-O2', '-g', '-std=c++17', '-Wall', '-fPIC', '-c', src, '-o', obj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, t) for t in tasks]:
            f.result()
    out = []
    for name, srcs in HOST_BINS.items():
        exe = os.path.join(BIN, name)
        deps = [objs[s] for s in HOST_COMMON + srcs] + [ENGINE_SO]
        if _stale(exe, deps):
            _run(['g++', '-o', exe] + [objs[s] for s in srcs + HOST_COMMON] +
                 [ENGINE_SO, '-Wl,-rpath,$ORIGIN/..', '-rdynamic', '-ldl', '-lpthread'])
        out.append(exe)
    # the formatter alone (no engine, no GPU): libaero_host.so
    so = os.path.join(BIN, 'libaero_host.so')
    capi = os.path.join(HOST, 'host_capi.cpp')
    if _stale(so, [capi, objs['qstr.cpp'], objs['output.cpp']] + hdrs):
        _run(['g++', '-O2', '-std=c++17', '-Wall', '-fPIC', '-shared', '-o', so, capi, objs['qstr.cpp'],
              objs['output.cpp']])
    out.append(so)
    for name, src in TOOL_BINS.items():
        exe = os.path.join(ROOT, 'tools', name)
        if _stale(exe, [src, os.path.join(HOST, 'zmq_dl.cpp'), os.path.join(HOST, 'zmq_dl.h')]):
            _run(['g++', '-O2', '-std=c++17', '-Wall', '-I', HOST, '-o', exe, src, objs['zmq_dl.cpp'], '-ldl'])
        out.append(exe)
    return out


# AddressSanitizer + UndefinedBehaviorSanitizer builds of every host-compiled
# source the CPU tests load: the oracle, the synthetic
# transmitter, the device libm's host build, the engine's host C++
# (acars_host, tables_host through tools/hostcheck.cpp) and the drop-in host
# binaries.  Host code only (no GPU sanitizer on this pool); tests/asan_check.sh
# runs the CPU tests against them.
ASAN_DIR = os.path.join(BUILD, 'asan')
SAN = ['-fsanitize=address,undefined', '-fno-sanitize-recover=undefined', '-fno-omit-frame-pointer', '-g']


def build_asan(jobs=4):
    d = ASAN_DIR
    bindir = os.path.join(d, 'bin')
    os.makedirs(bindir, exist_ok=True)
    base = ['g++', '-O1', '-std=c++17', '-fPIC'] + FP + SAN
    out = {}
    jobsl = []
    def lib(name, srcs, extra=()):
        so = os.path.join(d, name)
        out[name] = so
        if _stale(so, srcs + [os.path.join(CSRC, 'aero_math.h'), os.path.join(CSRC, 'aero_glibc_tables.h')]):
            jobsl.append(base + list(extra) + ['-shared', '-o', so] + srcs + ['-lm'])
    lib('liboracle.so', [os.path.join(ORACLE_DIR, 'aero_oracle.cpp'), os.path.join(ORACLE_DIR, 'pub_oracle.cpp')])
    lib('libaero_synth.so', [os.path.join(ROOT, 'tools', 'aero_synth.cpp')])
    lib('libaero_mathhost.so', [os.path.join(ROOT, 'tools', 'mathhost.cpp')])
    lib('libaero_hostcheck.so', HOSTCHECK_SRCS)
    hs = [os.path.join(HOST, s) for s in HOST_COMMON]
    lib(os.path.join('bin', 'libaero_host.so'), [os.path.join(HOST, 'host_capi.cpp')] + hs[:2])
    for name, srcs in HOST_BINS.items():
        exe = os.path.join(bindir, name)
        out[name] = exe
        allsrc = [os.path.join(HOST, s) for s in srcs] + hs
        if _stale(exe, allsrc + [ENGINE_SO]):
            jobsl.append(base + ['-o', exe] + allsrc + [ENGINE_SO, '-Wl,-rpath,' + HERE, '-rdynamic', '-ldl',
                                                          '-lpthread'])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, t) for t in jobsl]:
            f.result()
    return out


def build_all(jobs=4):
    build_oracle()
    build_synth()
    build_mathhost()
    build_fftsim()
    build_hostcheck()
    so = build_engine(jobs)
    build_diag(jobs)
    build_host(jobs)
    return so


# Diagnostic builds the GPU tests load (never the product): the demod's wave
# hand-off broken on purpose (tests/test_gpu_handoff.py)
DIAG_VARIANTS = {'handoff_fail': ['AERO_X_HANDOFF_FAIL']}


def build_diag(jobs=4):
    return [build_engine(jobs, variant=v, defines=d) for v, d in DIAG_VARIANTS.items()]


# Timing / traffic-attribution builds (not bit-exact, never loaded by a test):
# the demod without one buffer's accesses (scripts/pmc_demod_buffers.sh)
DROP_VARIANTS = {'drop%d' % k: ['AERO_X_DROP=%d' % k] for k in (1, 2, 4, 8)}


def build_drop(jobs=4):
    return [build_engine(jobs, variant=v, defines=d) for v, d in DROP_VARIANTS.items()]


# the burst demods with the general libm forms (same results; scripts/gpu_steps.sh ab=blibmK:burst10500)
BLIBM_VARIANTS = {'blibm%d' % k: ['AERO_X_BURST_LIBM=%d' % k] for k in (1, 2, 3)}


def build_blibm(jobs=4):
    return [build_engine(jobs, variant=v, defines=d) for v, d in BLIBM_VARIANTS.items()]


# the coarse kernel with every CIS gather on one line / without the y
# history reads (what each costs: scripts/gpu_steps.sh ab=cisline:oqpsk10500)
COARSE_VARIANTS = {'cisline': ['AERO_X_CISLINE'], 'noyread': ['AERO_X_NOYREAD']}


def build_coarse(jobs=4):
    return [build_engine(jobs, variant=v, defines=d) for v, d in COARSE_VARIANTS.items()]


# per-section s_memtime totals of the coarse kernel, the demod chain and the
# Viterbi (scripts/coarse_stamps.py, scripts/demod_stamps.py)
def build_stamps(jobs=4):
    return [build_engine(jobs, variant='stamps', defines=['AERO_X_STAMPS'])]


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--engine', action='store_true')
    ap.add_argument('--synth', action='store_true')
    ap.add_argument('--oracle', action='store_true')
    ap.add_argument('--host', action='store_true')
    ap.add_argument('--asan', action='store_true', help='sanitizer builds into build/asan (tests/asan_check.sh)')
    ap.add_argument('--variants', default='', help='comma list of timing builds: drop, blibm, coarse, stamps')
    ap.add_argument('-j', type=int, default=4)
    a = ap.parse_args()
    for v in filter(None, a.variants.split(',')):
        print({'drop': build_drop, 'blibm': build_blibm, 'coarse': build_coarse, 'stamps': build_stamps}[v](a.j))
    if a.asan:
        print(build_asan(a.j))
        sys.exit(0)
    if not (a.engine or a.synth or a.oracle or a.host):
        print(build_all(a.j))
        sys.exit(0)
    if a.oracle:
        print(build_oracle())
    if a.synth:
        print(build_synth())
    if a.engine:
        print(build_engine(a.j))
    if a.host:
        print(build_host(a.j))
