"""A ``dict`` whose values are built on first access (SURVEY §7 hard part 8).

``Environment.get_obs`` / ``step`` return ``Dict[int, EnvironmentObsDict]`` — one 21-key dict plus
nb_comm message dicts per house (environment.py:110-130).  At 1M houses building all of them is
seconds of Python per tick, though most callers read a few houses or go through the tensor API.
``LazyDict`` is a real ``dict`` subclass over a fixed key range: ``obs[k]``, iteration, ``len``,
``keys/values/items``, ``pd.DataFrame(obs)``, ``json.dumps``, ``copy.deepcopy``, pickling and
mutation behave as on the eager dict (the caller owns it and may mutate it); an entry is built from
the snapshot the environment took at ``get_obs`` time, the first time it is read.
"""
from __future__ import annotations

import copy
from collections.abc import ItemsView, KeysView, ValuesView


class LazyDict(dict):
    """``{k: build(k) for k in keys}``, each value built (once) when first read."""

    __slots__ = ("_build", "_keys", "_full")

    def __init__(self, build, keys: range):
        super().__init__()
        self._build = build
        self._keys = keys
        self._full = False
        if len(keys):  # one real entry: C-level emptiness checks (json's fast path) see a non-empty dict
            dict.__setitem__(self, keys[0], build(keys[0]))

    # ---------------------------------------------------------------- reads
    def __getitem__(self, k):
        try:
            return dict.__getitem__(self, k)
        except KeyError:
            if self._full or k not in self._keys:
                raise
            v = self._build(k)
            dict.__setitem__(self, k, v)
            return v

    def get(self, k, default=None):
        try:
            return self[k]
        except (KeyError, TypeError):
            return default

    def __contains__(self, k) -> bool:
        return dict.__contains__(self, k) if self._full else (k in self._keys)

    def __iter__(self):
        return dict.__iter__(self) if self._full else iter(self._keys)

    def __len__(self) -> int:
        return dict.__len__(self) if self._full else len(self._keys)

    def keys(self):
        return dict.keys(self) if self._full else KeysView(self)

    def values(self):
        return dict.values(self) if self._full else ValuesView(self)

    def items(self):
        return dict.items(self) if self._full else ItemsView(self)

    def __reversed__(self):
        return reversed(list(self.keys()))

    # ---------------------------------------------------------------- materialisation
    def materialize(self) -> "LazyDict":
        """Build every entry (in key order); from then on this is an ordinary dict."""
        if not self._full:
            items = [(k, self[k]) for k in self._keys]
            dict.clear(self)
            dict.update(self, items)
            self._full = True
        return self

    def __eq__(self, other):
        return dict.__eq__(self.materialize(), other)

    def __ne__(self, other):
        return not self == other

    __hash__ = None

    def __repr__(self) -> str:
        return dict.__repr__(self.materialize())

    def copy(self) -> dict:
        return dict(self.materialize())

    def __copy__(self) -> dict:
        return self.copy()

    def __deepcopy__(self, memo):
        return copy.deepcopy(dict(self.materialize()), memo)

    def __reduce_ex__(self, protocol):
        return (dict, (list(self.materialize().items()),))

    def __or__(self, other):
        return dict(self.materialize()) | other

    # ---------------------------------------------------------------- mutation: eager from here on
    def __setitem__(self, k, v):
        dict.__setitem__(self.materialize(), k, v)

    def __delitem__(self, k):
        dict.__delitem__(self.materialize(), k)

    def pop(self, *a):
        return dict.pop(self.materialize(), *a)

    def popitem(self):
        return dict.popitem(self.materialize())

    def setdefault(self, *a):
        return dict.setdefault(self.materialize(), *a)

    def update(self, *a, **kw):
        dict.update(self.materialize(), *a, **kw)

    def clear(self):
        self._full = True
        dict.clear(self)

    def __ior__(self, other):
        self.update(other)
        return self
