"""Every DTC_* switch the sources read is listed in docs/KNOBS.md (and nothing stale is listed)."""

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_training_compare_jax_amd")

# environment reads (Python os.environ / C getenv) and compile-time switches (#ifdef / #ifndef)
_READ = [re.compile(r'environ(?:\.get)?\(\s*"(DTC_[A-Z0-9_]+)"'),
         re.compile(r'environ\[\s*"(DTC_[A-Z0-9_]+)"\s*\]'),
         re.compile(r'getenv\(\s*"(DTC_[A-Z0-9_]+)"'),
         re.compile(r'#\s*if(?:n?def)\s+(DTC_[A-Z0-9_]+)')]
# header guards / helpers that are code, not switches
_NOT_SWITCHES = {"DTC_CHECK_LAUNCH", "DTC_LDS", "DTC_OUT_STORE", "DTC_NV_SWITCH", "DTC_WAVE", "DTC_ASSERT",
                 "DTC_HOST_CHECK"}


def _sources():
    for base, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                yield os.path.join(base, f)
    yield os.path.join(ROOT, "bench.py")


def _switches_read():
    found = {}
    for path in _sources():
        with open(path, encoding="utf-8", errors="replace") as fh:
            text = fh.read()
        for rx in _READ:
            for name in rx.findall(text):
                if name not in _NOT_SWITCHES:
                    found.setdefault(name, os.path.relpath(path, ROOT))
    return found


def _documented():
    with open(os.path.join(ROOT, "docs", "KNOBS.md"), encoding="utf-8") as fh:
        return set(re.findall(r"`(DTC_[A-Z0-9_]+)`", fh.read()))


def test_every_switch_is_documented():
    missing = {k: v for k, v in _switches_read().items() if k not in _documented()}
    assert not missing, f"undocumented DTC_* switches (add them to docs/KNOBS.md): {missing}"


def test_no_stale_entries():
    stale = _documented() - set(_switches_read()) - _NOT_SWITCHES
    assert not stale, f"docs/KNOBS.md lists switches nothing reads: {sorted(stale)}"
