"""pytest plugin for A/B runs of the GPU tests on an alternate kernel: every SirenEngine gets cfg.reserved |= the
integer in SIREN_TEST_FLAGS (e.g. 4 = SIREN_FLAG_W3_SERIAL). Usage: python -m pytest -p tools.flags_plugin ..."""
import os


def pytest_configure(config):
    flags = int(os.environ.get('SIREN_TEST_FLAGS', '0'))
    if not flags:
        return
    from siren_amd import engine as E
    init = E.SirenEngine.__init__

    def patched(self, *a, **k):
        k['flags'] = int(k.get('flags', 0)) | flags
        init(self, *a, **k)
    E.SirenEngine.__init__ = patched
