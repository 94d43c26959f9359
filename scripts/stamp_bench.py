"""bench.write_stamp_leg on its own (one GPU): flush-batch trailers stamped by rh_crc32c_stamp_host
(PCIe included) against the oracle's PureJavaCrc32C on one core, 16 KiB .. 8 MiB.

    python scripts/stamp_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from ratis_amd import engine
    ctx = engine.Context(0)
    print(json.dumps({"write_stamp": bench.write_stamp_leg(ctx)}))


if __name__ == "__main__":
    main()
