"""experimental.shuffle (reference python/ray/experimental/shuffle.py; its driver is what the
reference's shuffle scalability tests run): every item of every input partition lands in exactly
one output partition, for the streaming (refs) and non-streaming writers, a custom partitioner,
and the CLI driver with the store forced to spill."""
import numpy as np

import ray_community_amd as ray
from ray_community_amd.experimental import shuffle


def _reader(i):
    for k in range(12):
        yield (i, k)


def test_simple_shuffle_routes_every_item_once(shutdown_only):
    ray.init(num_cpus=4)

    def writer(j, refs):
        return sorted(ray.get(refs))

    out = shuffle.simple_shuffle(input_reader=_reader, input_num_partitions=5, output_num_partitions=3,
                                 output_writer=writer)
    assert len(out) == 3
    seen = [x for part in out for x in part]
    assert sorted(seen) == sorted((i, k) for i in range(5) for k in range(12))
    # round robin: item k of every input went to partition k % 3
    for j, part in enumerate(out):
        assert all(k % 3 == j for _i, k in part)

    out2 = shuffle.simple_shuffle(input_reader=_reader, input_num_partitions=5, output_num_partitions=3,
                                  output_writer=lambda j, items: sorted(items),
                                  object_store_writer=shuffle.ObjectStoreWriterNonStreaming)
    assert out2 == out

    def by_input(stream, n):  # custom partitioner: route by the input partition id
        for item in stream:
            yield item[0] % n, item

    seen = []
    out3 = shuffle.simple_shuffle(input_reader=_reader, input_num_partitions=4, output_num_partitions=2,
                                  output_writer=lambda j, items: sorted(items), partitioner=by_input,
                                  object_store_writer=shuffle.ObjectStoreWriterNonStreaming,
                                  progress=lambda t: seen.append(t.poll()))
    assert {i for i, _ in out3[0]} == {0, 2} and {i for i, _ in out3[1]} == {1, 3}
    assert seen[-1] == (4 * 2, 2)  # every map output and every reduce finished

    one = shuffle.simple_shuffle(input_reader=_reader, input_num_partitions=2, output_num_partitions=1,
                                 output_writer=lambda j, refs: len(refs))
    assert one == [24]


def test_shuffle_driver_moves_every_byte_through_a_small_store(shutdown_only):
    # 4 x 4 partitions of 3 MB in 1 MB rows through a 16 MB store: large rows go to the shm
    # store and are spilled / restored as it fills
    stats = shuffle.run(num_partitions=4, partition_size=3e6, num_cpus=4, object_store_memory=16e6, use_wait=True)
    assert stats["shuffled_bytes"] == 4 * 3_000_000
    assert not ray.is_initialized()  # the driver shut the session it started down
    stats = shuffle.run(num_partitions=3, partition_size=2e6, num_nodes=2, num_cpus=2, object_store_memory=64e6,
                        no_streaming=True)
    assert stats["shuffled_bytes"] == 3 * 2_000_000
    assert np.isfinite(stats["mb_per_s"])
