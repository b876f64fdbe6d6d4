"""Host-resident rates (bench.py host_resident: tickets and the stream mirror)
with the zero-copy row moves on and off (rs_debug_set_path("zc", v))."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    import reedsolomon16_amd as rs
    from reedsolomon16_amd import _capi

    for rep in range(2):
        for v in (0, 3):
            _capi.set_path("zc", v)
            r = bench.host_resident(rs)
            print(json.dumps({"zc": v, "rep": rep, "tickets": r["tickets"], "stream": r["stream"], "stream_threads8": r.get("stream_threads8")}), flush=True)
    _capi.reset_paths()


if __name__ == "__main__":
    main()
