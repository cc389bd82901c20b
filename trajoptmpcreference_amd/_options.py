"""The empty-options default of the reference's signatures.

The reference writes ``options={}`` as the default of many methods and fills that
dict in place with ``setdefault`` (TrajoptMPCReference.py:91-115, TrajoptPlant.py:29-34,
PCG.py:19-25), so one call's defaults leak into the next.  Here the
default is NO_OPTIONS: an empty dict, equal to the reference's ``{}`` (the signatures
match, tests/test_signatures.py), that raises if anything tries to fill it.  Every
method that accepts it starts with ``options = fresh(options)``.
"""


class _FrozenEmpty(dict):
    def _refuse(self, *args, **kwargs):
        raise TypeError("the shared default options dict is read-only (pass your own dict to receive the defaults)")

    __setitem__ = __delitem__ = setdefault = update = pop = popitem = clear = _refuse


NO_OPTIONS = _FrozenEmpty()


def fresh(options):
    """A new dict for the default, the caller's own dict (filled in place, as the reference) otherwise."""
    if options is NO_OPTIONS or options is None:
        return {}
    return options
