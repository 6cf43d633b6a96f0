"""CPU check that the boundary's documentation matches what the measurement reads: every kernel /
counter name bench.py asks lsm_kernel_stats for is listed in include/lidarsm.h's instrumentation
comment, and every name that comment lists is one the library records (csrc tic / stats)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _header_stats_comment():
    h = _read("include", "lidarsm.h")
    a = h.index("/* Instrumentation")
    return h[a:h.index("*/", a)]


def _bench_names():
    src = _read("bench.py")
    names = set(re.findall(r'(?:kstats|kernel_stats)\("([a-z0-9_]+)"\)', src))
    m = re.search(r"^KERNELS = \[(.*?)\]", src, re.S | re.M)
    names |= set(re.findall(r'"([a-z0-9_]+)"', m.group(1)))
    m = re.search(r'kstats\(k\)\["launches"\] for k in \((.*?)\)', src, re.S)
    names |= set(re.findall(r'"([a-z0-9_]+)"', m.group(1)))
    return names


def _library_names():
    names = set()
    csrc = os.path.join(ROOT, "lidar_slam_arvc_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            s = _read("lidar_slam_arvc_amd", "csrc", f)
            names |= set(re.findall(r'tic\("([a-z0-9_]+)"', s))
            names |= set(re.findall(r'stats\["([a-z0-9_]+)"\]', s))
            # loops over names: for (const char *k : {"nn", "nn_fallback"})
            for grp in re.findall(r'for \(const char \*k : \{([^}]*)\}\)', s):
                names |= set(re.findall(r'"([a-z0-9_]+)"', grp))
    return names


def test_bench_stats_names_documented():
    doc = _header_stats_comment()
    listed = set(re.findall(r'"([a-z0-9_]+)"', doc))
    missing = sorted(_bench_names() - listed)
    assert not missing, f"bench.py reads stats the header does not document: {missing}"


def test_documented_stats_names_exist():
    doc = _header_stats_comment()
    listed = set(re.findall(r'"([a-z0-9_]+)"', doc))
    stale = sorted(listed - _library_names())
    assert not stale, f"include/lidarsm.h documents stats the library never records: {stale}"
