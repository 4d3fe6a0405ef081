"""Load the reference's analysis modules (utils, classes) under Python 3 — survey container only.

This is golden-vector tooling, not product code and not an oracle restatement: it imports the
upstream reference from /root/reference (read-only) with stub `boto`/`osgeo` modules and four
line-preserving token substitutions for Python-2 idioms. Nothing from the
reference is copied into the repository; only the numeric outputs it produces are committed as
fixtures under tests/golden/. /root/reference does not exist on the GPU box: nothing that runs
there imports this file.
"""
import re
import sys
import types
import warnings

REF = '/root/reference'
_SUBS = [(r'\.iteritems\(\)', '.items()'), (r'\bxrange\(', 'range('),
         (r'it\.next\(\)', 'next(it)'), (r'\bunicode\(self\)', 'str(self)')]


def load_reference():
    """Return (utils, classes) modules of the reference, loaded with the Appendix C shim."""
    if 'classes' in sys.modules and getattr(sys.modules['classes'], '_lt_ref', False):
        return sys.modules['utils'], sys.modules['classes']
    boto = types.ModuleType('boto')

    def _no_s3(*a, **k):
        raise RuntimeError('S3 disabled in golden generation')
    boto.connect_s3 = _no_s3
    sys.modules['boto'] = boto
    osgeo = types.ModuleType('osgeo')
    osgeo.gdal = types.ModuleType('osgeo.gdal')
    osgeo.ogr = types.ModuleType('osgeo.ogr')
    sys.modules.update({'osgeo': osgeo, 'osgeo.gdal': osgeo.gdal, 'osgeo.ogr': osgeo.ogr})
    if REF not in sys.path:
        sys.path.insert(0, REF)
    warnings.filterwarnings('ignore', category=FutureWarning)
    warnings.filterwarnings('ignore', category=DeprecationWarning)
    mods = {}
    for name in ['classes', 'utils']:
        path = '%s/%s.py' % (REF, name)
        src = open(path).read()
        for pat, rep in _SUBS:
            src = re.sub(pat, rep, src)
        mod = types.ModuleType(name)
        mod.__file__ = path
        mod._lt_ref = True
        sys.modules[name] = mod
        exec(compile(src, path, 'exec'), mod.__dict__)
        mods[name] = mod
    return mods['utils'], mods['classes']
