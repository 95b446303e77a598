import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mri-to-speech_amd")
# the plug-in directory is what --mri-code-dir puts on sys.path (run_mri_video_inference.py:119-126)
for p in (os.path.join(PKG, "mri2speech_code"), PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libm2s.so")
