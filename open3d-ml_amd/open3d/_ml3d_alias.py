"""The Open3D-ML half of the ``open3d.ml`` namespace.

Upstream Open3D bundles Open3D-ML and, when ``OPEN3D_ML_ROOT`` names a
checkout, imports that checkout's ``ml3d`` instead (the reference's
``set_open3d_ml_root.sh:3``, ``docs/howtos.md:235-245``, ``README.md:313-316``):
``open3d.ml.{configs,datasets,utils,vis}`` and
``open3d.ml.torch.{dataloaders,models,modules,pipelines}`` are ``ml3d``'s
packages, so ``import open3d.ml.torch as ml3d; ml3d.models.RandLANet(...)``
(``tests/test_models.py:36-38``) builds the checkout's model, whose own
``open3d.ml.torch.ops`` / ``layers`` / ``contrib`` imports land on this
build's HIP ops.

This shim bundles no Open3D-ML copy: the ``ml3d`` package comes from
``OPEN3D_ML_ROOT`` (appended to ``sys.path`` by ``open3d/__init__.py``, as
upstream) or from ``sys.path`` as it is.  The names resolve lazily
(``__getattr__`` on the two namespace modules) and as real submodules
(``import open3d.ml.torch.models`` / ``from open3d.ml.torch.models import X``
through a meta-path alias), so importing ``open3d.ml.torch`` never imports the
model zoo, datasets or the GUI visualiser unless they are used.
"""
import importlib
import importlib.abc
import importlib.util
import sys

# open3d name -> ml3d module (upstream open3d/ml/__init__.py and
# open3d/ml/torch/__init__.py import exactly these)
ML_NAMES = ("configs", "datasets", "utils", "vis")
TORCH_NAMES = ("dataloaders", "models", "modules", "pipelines")
ALIASES = {f"open3d.ml.{n}": f"ml3d.{n}" for n in ML_NAMES}
ALIASES.update({f"open3d.ml.torch.{n}": f"ml3d.torch.{n}" for n in TORCH_NAMES})
# upstream also puts configs / datasets / utils / vis next to the torch names
ALIASES.update({f"open3d.ml.torch.{n}": f"ml3d.{n}" for n in ML_NAMES})


def ml3d_available():
    try:
        return importlib.util.find_spec("ml3d") is not None
    except (ImportError, ValueError):
        return False


def target_of(fullname):
    """The ml3d module an ``open3d.ml[.torch].<name>[.<rest>]`` name stands
    for (whole subtrees: ``open3d.ml.torch.models.randlanet`` is
    ``ml3d.torch.models.randlanet``), or None."""
    for alias, target in ALIASES.items():
        if fullname == alias or fullname.startswith(alias + "."):
            return target + fullname[len(alias):]
    return None


class _Ml3dAlias(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Resolves ``open3d.ml[.torch].<name>`` and every module below it to the
    ``ml3d`` module itself (the same module object: no second copy, class
    registries shared).  The module keeps its own ``__spec__`` (importlib
    sets the alias spec on it; exec_module puts the original back)."""

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith("open3d.ml.") or target_of(fullname) is None or not ml3d_available():
            return None
        return importlib.util.spec_from_loader(fullname, self)

    def __init__(self):
        self._orig = {}  # id(module) -> its own (__spec__, __loader__)

    def create_module(self, spec):
        module = importlib.import_module(target_of(spec.name))
        self._orig[id(module)] = (module.__spec__, getattr(module, "__loader__", None))
        return module

    def exec_module(self, module):
        # already executed as ml3d.*; importlib has just set the alias spec
        # (no origin, no search locations) on it: put its own back
        orig = self._orig.pop(id(module), None)
        if orig is not None:
            module.__spec__, module.__loader__ = orig


def install():
    # ahead of the path finders: a submodule of an aliased package (whose
    # __path__ is the ml3d directory) would otherwise be loaded a second time
    # under the open3d name
    if not any(isinstance(f, _Ml3dAlias) for f in sys.meta_path):
        sys.meta_path.insert(0, _Ml3dAlias())


def module_getattr(namespace, name):
    """``__getattr__`` body of the namespace modules."""
    full = f"{namespace}.{name}"
    if full not in ALIASES:
        raise AttributeError(f"module {namespace!r} has no attribute {name!r}")
    if not ml3d_available():
        raise AttributeError(
            f"{full} is Open3D-ML's {ALIASES[full]}: set OPEN3D_ML_ROOT to an Open3D-ML checkout "
            f"(source set_open3d_ml_root.sh) or put its ml3d package on sys.path")
    return importlib.import_module(full)
