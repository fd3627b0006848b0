"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's algorithm for the hot path (tier_r) and of the
build-defined north_star operators (tier_n, parity unpinned by the reference).  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import it, and only as the checker / CPU baseline.  The product package
(``lidar_ai_recommendation_software_amd``) never imports it.
"""
