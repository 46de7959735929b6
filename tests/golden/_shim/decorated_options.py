"""Minimal local stand-in for the third-party ``decorated_options`` package.

The reference imports ``decorated_options`` (utils.py:12, opt_runs.py:5) for
``Options`` bundles and the ``@optioned`` kwarg-injection decorator.  The package
is not installed in this image and there is no network, so the golden-fixture
generator puts this file on ``sys.path`` before importing the reference.  Only
the behaviour the reference's call sites rely on is provided.
"""
import functools
import inspect


class Options:
    def __init__(self, **kw):
        self.__dict__.update(kw)

    def set_new(self, **kw):
        d = dict(self.__dict__)
        d.update(kw)
        return Options(**d)

    def set(self, **kw):
        return self.set_new(**kw)

    def _get_dict(self):
        return dict(self.__dict__)

    def __repr__(self):
        return "Options(%r)" % (self.__dict__,)


def optioned(option_arg="opts"):
    def deco(fn):
        sig = inspect.signature(fn)

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            opts = kwargs.get(option_arg)
            if option_arg not in sig.parameters:
                kwargs.pop(option_arg, None)
            if opts is not None:
                bound = sig.bind_partial(*args, **kwargs)
                for name in sig.parameters:
                    if name == option_arg or name in bound.arguments:
                        continue
                    if hasattr(opts, name):
                        kwargs[name] = getattr(opts, name)
            return fn(*args, **kwargs)

        return wrapper

    return deco
