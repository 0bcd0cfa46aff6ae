"""Import helper: the package directory name carries hyphens (not a Python
identifier), so it is registered as ``hvit_amd``.

    import hvit_amd_loader; hvit = hvit_amd_loader.load()
    model = hvit.HybridViT().cuda()
"""

import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "speech-enhancement-via-hybrid-vision-transformer-project_amd")
NAME = "hvit_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
