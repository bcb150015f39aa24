"""Import shim for the product package, whose directory name
(``ruleset-analysis_amd``) is not a Python identifier.  ``load()`` registers it
as ``ruleset_analysis_amd`` so ``import ruleset_analysis_amd.engine`` works."""

import importlib.util
import os
import sys

NAME = 'ruleset_analysis_amd'
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ruleset-analysis_amd')


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(ROOT, '__init__.py'),
                                                  submodule_search_locations=[ROOT])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
