"""Native placement-group directory (``_native/pg_table.cpp``): records, name index, pending FIFO
and state counts the head's placement-group RPCs use."""
import pytest

from ray_community_amd._private.object_store import native


def test_pg_directory_lifecycle():
    d = native().PgDirectory()
    a, b = b"\x01" * 18, b"\x02" * 18
    d.add(a, "grp", "PACK", [{"CPU": 1.0}, {"CPU": 2.0}], None, 1.0, False)
    d.add(b, "", "SPREAD", [{"GPU": 1.0}], "detached", 2.0, True)
    assert len(d) == 2 and a in d and b"\x03" * 18 not in d
    assert d.state(a) == "PENDING" and d.state(b"\x03" * 18) == ""
    assert d.pending() == [a, b]                      # creation order
    assert d.by_name("grp") == a and d.by_name("nope") is None
    assert d.infeasible(b) and not d.infeasible(a)
    assert d.nodes(a) is None
    d.set_nodes(a, ["n1", "n2"])
    d.set_state(a, "CREATED")                          # placed: leaves the pending queue
    assert d.pending() == [b] and d.nodes(a) == ["n1", "n2"]
    info = d.info(a)
    assert info == {"placement_group_id": a.hex(), "name": "grp", "strategy": "PACK", "state": "CREATED",
                    "bundles": {0: {"CPU": 1.0}, 1: {"CPU": 2.0}}, "bundles_to_node_id": {0: "n1", 1: "n2"}}
    assert set(d.table()) == {a.hex(), b.hex()} and d.info(b"\x03" * 18) == {}
    assert d.state_counts() == {"CREATED": 1, "PENDING": 1}
    d.set_state(a, "REMOVED")
    assert d.by_name("grp") is None                    # a removed group frees its name
    d.set_state(b, "REMOVED")
    assert d.pending() == [] and d.state_counts() == {"REMOVED": 2}
    with pytest.raises(ValueError):
        d.add(a, "x", "PACK", [], None, 0.0, False)
    with pytest.raises(KeyError):
        d.set_state(b"\x04" * 18, "CREATED")
