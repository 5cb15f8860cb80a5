"""Host-side logic of the plugin mirror that needs no device (pyrope_amd/vector.py)."""
import pytest


def test_get_int_param_semantics():  # VectorIndexRegistry.cs:115-126 GetIntParam
    from pyrope_amd import VectorIndexRegistry
    from pyrope_amd._lib import FormatException
    f = VectorIndexRegistry._int_param
    assert f(None, "nlist", 100) == 100
    assert f({}, "nlist", 100) == 100
    assert f({"nlist": 500}, "nlist", 100) == 500
    assert f({"nlist": "250"}, "nlist", 100) == 250        # int.TryParse on strings
    assert f({"nlist": " -7 "}, "nlist", 100) == -7
    assert f({"nlist": "+12"}, "nlist", 100) == 12
    assert f({"nlist": "1_000"}, "nlist", 100) == 100      # TryParse rejects separators
    assert f({"nlist": "abc"}, "nlist", 100) == 100
    assert f({"nlist": "99999999999"}, "nlist", 100) == 100  # Int32 overflow -> TryParse false
    assert f({"nlist": True}, "nlist", 100) == 100         # JSON true is not a Number
    assert f({"nlist": 64.0}, "nlist", 100) == 64
    assert f({"nlist": None}, "nlist", 100) == 100
    with pytest.raises(FormatException):
        f({"nlist": 3.5}, "nlist", 100)                    # GetInt32 on a non-integral number
    with pytest.raises(FormatException):
        f({"nlist": 2**40}, "nlist", 100)


def test_search_options_defaults():  # SearchOptions.cs:3
    from pyrope_amd import SearchOptions
    o = SearchOptions()
    assert o.max_scans is None and o.nprobe is None and o.ef_search is None


def test_labels_never_collide_after_caller_chosen_labels():
    """a new id must not get a label already handed out through add_labels
    (e.g. the sparse shard labels r, r + world, ...)."""
    import numpy as np

    from pyrope_amd.vector import HipVectorIndex
    ix = object.__new__(HipVectorIndex)  # host bookkeeping only: no device handle
    ix._label_of, ix._id_of, ix._next_label = {}, {}, 0
    ix._register_labels(np.array([1, 3, 5, 7], np.int64))
    new = [ix._label("a"), ix._label("b"), ix._label("a")]
    assert new == [8, 9, 8]
    assert set(new).isdisjoint({1, 3, 5, 7})
    ix._register_labels(np.array([2], np.int64))  # lower than the counter: the counter keeps going
    assert ix._label("c") == 10
    assert ix._id_of[8] == "a" and ix._label_of["7"] == 7



def test_sq_span_overload_throws_on_length_mismatch():  # ScalarQuantizerTests.cs:62-68
    import numpy as np
    import pytest

    from pyrope_amd import ArgumentException, ScalarQuantizer
    with pytest.raises(ArgumentException, match="lengths must match"):
        ScalarQuantizer.quantize_into(np.zeros(2, np.float32), np.zeros(3, np.uint8))
    assert ScalarQuantizer.quantize([]) [1:] == (0.0, 0.0)  # empty vector: min = max = 0, no device call
