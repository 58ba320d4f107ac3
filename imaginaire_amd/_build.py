"""Native build for the gfx950 HIP extension ``imaginaire_amd._C``.

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` (no
hipify pass, no CUDA sources: the kernels are written in HIP for CDNA4), the
host-only binding ``csrc/bindings.cpp`` by the host C++ compiler, and the
objects are linked into ``imaginaire_amd/_C.so`` in-tree so the shared object
travels with the repository snapshot to the GPU box.

Usage: ``python -m imaginaire_amd._build [-j N] [--force]``.
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(os.path.dirname(HERE), 'build', 'csrc')
TARGET = os.path.join(HERE, '_C.so')
# provenance of the in-tree _C.so: arch, digest of every csrc source, compiler, build mode
MANIFEST = os.path.join(HERE, '_C.build.json')
ARCH = os.environ.get('IMAGINAIRE_AMD_ARCH', 'gfx950')


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, 'include'),
           os.path.join(root, 'include', 'torch', 'csrc', 'api', 'include')]
    lib = os.path.join(root, 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _common_flags():
    inc, _, abi = _torch_paths()
    flags = ['-O3', '-fPIC', '-std=c++17',
             '-DTORCH_EXTENSION_NAME=_C', '-DTORCH_API_INCLUDE_EXTENSION_H',
             '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-DUSE_ROCM=1',
             '-I' + CSRC, '-I' + sysconfig.get_paths()['include'],
             '-Wno-unused-result', '-Wno-deprecated-declarations']
    for p in inc:
        flags += ['-isystem', p]
    return flags


def _hipcc():
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    return os.path.join(rocm, 'bin', 'hipcc')


def _sources():
    hip = sorted(f for f in os.listdir(CSRC) if f.endswith('.hip'))
    cpp = sorted(f for f in os.listdir(CSRC) if f.endswith('.cpp'))
    return hip, cpp


def _headers_digest():
    h = hashlib.sha1()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(('.h', '.hpp', '.cuh', '.inc')):
            with open(os.path.join(CSRC, f), 'rb') as fh:
                h.update(fh.read())
    return h.hexdigest()[:12]


def sources_digest():
    """sha1 over every csrc source and header (name + bytes): identifies the code a _C.so
    was built from (checked at import by ``ops/_ext.py``)."""
    h = hashlib.sha1()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(('.hip', '.cpp', '.h', '.hpp', '.inc')):
            h.update(f.encode())
            with open(os.path.join(CSRC, f), 'rb') as fh:
                h.update(fh.read())
    return h.hexdigest()


def _hipcc_version():
    try:
        r = subprocess.run([_hipcc(), '--version'], capture_output=True, text=True, timeout=60)
        lines = [ln for ln in r.stdout.splitlines() if 'version' in ln.lower()]
        return lines[0].strip() if lines else r.stdout.strip()[:120]
    except Exception as e:  # noqa: BLE001
        return 'unknown (%s)' % e


def _code_object_archs(path):
    """gfx targets embedded in a shared object's offload bundle (``--offload-arch``)."""
    import re
    with open(path, 'rb') as f:
        blob = f.read()
    return sorted(set(m.decode() for m in re.findall(rb'amdgcn-amd-amdhsa--(gfx[0-9a-f]+)', blob)))


def _write_manifest(mode, n_sources, compiled):
    import json
    import time
    info = {'arch': ARCH, 'code_object_archs': _code_object_archs(TARGET),
            'sources_sha1': sources_digest(), 'n_sources': n_sources,
            'recompiled_objects': compiled, 'mode': mode, 'hipcc': _hipcc_version(),
            'built_at': time.strftime('%Y-%m-%dT%H:%M:%SZ', time.gmtime())}
    with open(MANIFEST + '.tmp', 'w') as f:
        json.dump(info, f, indent=1)
    os.replace(MANIFEST + '.tmp', MANIFEST)
    return info


def _compile(src, force, hdr):
    path = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, src + '.' + hdr + '.o')
    if not force and os.path.exists(obj) and \
            os.path.getmtime(obj) >= os.path.getmtime(path):
        return obj, 'cached'
    if src.endswith('.hip'):
        cmd = [_hipcc(), '-x', 'hip', '--offload-arch=' + ARCH,
               '-munsafe-fp-atomics', '-c', path, '-o', obj] + _common_flags()
    else:
        cxx = os.environ.get('CXX', 'g++')
        cmd = [cxx, '-c', path, '-o', obj] + _common_flags()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return None, 'compile failed: {}\n{}\n{}'.format(' '.join(cmd), r.stdout, r.stderr)
    return obj, 'compiled'


def build(jobs=None, force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    hip, cpp = _sources()
    hdr = _headers_digest()
    jobs = jobs or min(8, os.cpu_count() or 4)
    objs, errors, compiled = [], [], 0
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_compile, s, force, hdr): s for s in hip + cpp}
        for fut in cf.as_completed(futs):
            obj, status = fut.result()
            if obj is None:
                errors.append(status)
            else:
                objs.append(obj)
                compiled += status == 'compiled'
    if errors:
        raise RuntimeError('\n\n'.join(errors))
    newest = max(os.path.getmtime(o) for o in objs)
    if not force and os.path.exists(TARGET) and os.path.getmtime(TARGET) >= newest:
        info = _write_manifest('up-to-date', len(objs), compiled)
        if verbose:
            print('[imaginaire_amd._build] up to date: %s (archs %s, sources %s)' % (
                TARGET, ','.join(info['code_object_archs']), info['sources_sha1'][:12]))
        return TARGET
    _, lib, _ = _torch_paths()
    cmd = [_hipcc(), '-shared', '-fPIC', '--offload-arch=' + ARCH] + sorted(objs) + [
        '-L' + lib, '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip',
        '-ltorch_python', '-Wl,-rpath,' + lib,
        # RCCL is NOT linked: its nccl* symbols resolve at load time from the librccl.so that
        # libtorch_hip already depends on (torch/lib). Linking -lrccl recorded a NEEDED
        # librccl.so.1 that the loader found in /opt/rocm/lib — a second RCCL copy in the
        # process whose exit-time destructors corrupted the heap (abort at interpreter exit)
        '-o', TARGET + '.tmp']
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed: {}\n{}\n{}'.format(' '.join(cmd), r.stdout, r.stderr))
    # a host pass that silently drops a kernel's launch stub links fine and fails only at
    # import time (undefined __device_stub__ symbol): check the fresh object before publishing
    r2 = subprocess.run(['nm', '-u', '-C', TARGET + '.tmp'], capture_output=True, text=True)
    missing = [ln for ln in r2.stdout.splitlines() if '__device_stub__' in ln]
    if missing:
        raise RuntimeError('link produced undefined kernel stubs:\n' + '\n'.join(missing))
    os.replace(TARGET + '.tmp', TARGET)
    info = _write_manifest('linked', len(objs), compiled)
    if ARCH not in info['code_object_archs']:
        raise RuntimeError('%s holds code objects for %s, not %s' % (
            TARGET, info['code_object_archs'], ARCH))
    if verbose:
        print('[imaginaire_amd._build] built %s from %d sources (%d recompiled; archs %s, '
              'sources %s)' % (TARGET, len(objs), compiled, ','.join(info['code_object_archs']),
                               info['sources_sha1'][:12]))
    return TARGET


def main():
    p = argparse.ArgumentParser()
    p.add_argument('-j', type=int, default=None)
    p.add_argument('--force', action='store_true')
    a = p.parse_args()
    try:
        build(a.j, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)


if __name__ == '__main__':
    main()
