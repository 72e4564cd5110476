#!/bin/bash
# heavy-tile kernel variants on fsuzane 1080p x64 (BASELINE C3)
python tools/ab_frame.py --cfg scene='"fsuzane"' librtc.so
python tools/ab_frame.py --cfg scene='"fsuzane"' --cfg coop_lanes=4 librtc.so
python tools/ab_frame.py --cfg scene='"fsuzane"' --cfg pipe=true librtc.so
python tools/ab_frame.py --cfg scene='"fsuzane"' --cfg spec=true librtc.so
