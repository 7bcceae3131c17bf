"""CPU oracle of the reference hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, as the checker or the timed CPU baseline.  The product path (cfd_julia_amd,
libcfdj.so) never imports, links or calls it.  See vm_oracle.py for how it is pinned to
the reference's published numbers.
"""
