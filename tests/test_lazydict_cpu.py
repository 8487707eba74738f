"""LazyDict (the dict the drop-in Environment returns for obs / rewards) behaves like the eager
dict for the ways the reference's callers use it: indexing, iteration, len, keys/values/items,
pd.DataFrame(obs).transpose() (client_manager_service.py:159, greedy_myopic_controller.py:77),
copy.deepcopy (greedy_myopic_controller.py:57), json, pickle, mutation by the caller."""
import copy
import json
import pickle

import pandas as pd
import pytest

from mdr_amd.lazydict import LazyDict

N = 7


def _mk(counter):
    def build(k):
        counter.append(k)
        return {"indoor_temp": 20.0 + k, "turned_on": k % 2 == 0, "message": [{"x": k}]}

    return LazyDict(build, range(N))


def _eager():
    return {k: {"indoor_temp": 20.0 + k, "turned_on": k % 2 == 0, "message": [{"x": k}]} for k in range(N)}


def test_builds_on_access_only():
    built = []
    d = _mk(built)
    assert built == [0]  # one real entry (C-level emptiness checks)
    assert d[5]["indoor_temp"] == 25.0 and built == [0, 5]
    assert d[5] is d[5] and built == [0, 5]  # built once
    assert len(d) == N and 3 in d and N not in d and list(d) == list(range(N))
    assert built == [0, 5]
    with pytest.raises(KeyError):
        d[N]
    assert d.get(N, "x") == "x"


def test_matches_eager_dict_for_reference_callers():
    d, e = _mk([]), _eager()
    assert d == e and e == d.copy()
    assert list(d.keys()) == list(e.keys()) and list(d.values()) == list(e.values())
    assert list(d.items()) == list(e.items())
    pd.testing.assert_frame_equal(pd.DataFrame(_mk([])).transpose(), pd.DataFrame(e).transpose())
    assert json.dumps(_mk([])) == json.dumps(e)
    assert copy.deepcopy(_mk([])) == e and type(copy.deepcopy(_mk([]))) is dict
    assert pickle.loads(pickle.dumps(_mk([]))) == e
    assert dict(_mk([])) == e and {**_mk([])} == e


def test_caller_mutation():
    d = _mk([])
    d[3]["indoor_temp"] = -1.0  # mutating a built entry sticks
    assert d[3]["indoor_temp"] == -1.0
    d[99] = "extra"
    del d[0]
    assert len(d) == N and 99 in d and 0 not in d and d[3]["indoor_temp"] == -1.0
    assert d.pop(99) == "extra" and len(d) == N - 1
