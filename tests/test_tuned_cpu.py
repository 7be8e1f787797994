"""The shipped per-shape conv tile tables (models/tuned_tiles*_mi355x.json) load, with keys of the arity the
executors look up -- a table that silently failed to load would fall every shape back to the static tile rule
(~2 ms/step on ResNet-50) -- and a broken shipped table warns instead of passing quietly."""
import json
import warnings

import pytest


def test_shipped_tables_load_with_executor_key_arity():
    from pytorch_distributed_template_amd.models import tuned
    from pytorch_distributed_template_amd.models.executor import ResNetExecutor
    t16 = tuned.load_table(tuned.TABLE16, tuned.ARITY16)
    t32 = tuned.load_table(tuned.TABLE32, tuned.ARITY32)
    assert len(t16) >= 10 and len(t32) >= 5
    for k, v in t16.items():
        assert len(k) == tuned.ARITY16[k[0]]
        assert tuple(v) in ResNetExecutor._CANDIDATES, (k, v)
    for k, v in t32.items():
        assert len(k) == tuned.ARITY32[k[0]] and all(x > 0 for x in v)


def test_executor_module_tables_are_the_shipped_ones():
    from pytorch_distributed_template_amd.models import executor, tuned
    assert executor._TUNED == tuned.load_table(tuned.TABLE16, tuned.ARITY16)


@pytest.mark.parametrize("content", ["not json", json.dumps({"tiles": [[["fwd", 1, 2], [128, 128]]]}),
                                     json.dumps({"note": "no tiles"})])
def test_broken_shipped_table_warns(tmp_path, content):
    from pytorch_distributed_template_amd.models import tuned
    p = tmp_path / "t.json"
    p.write_text(content)
    with pytest.warns(RuntimeWarning, match="could not be loaded"):
        assert tuned.load_table(str(p), tuned.ARITY16) == {}
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert tuned.load_table(str(p), tuned.ARITY16, shipped=False) == {}  # user tables: no warning
