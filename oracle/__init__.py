"""TEST INFRASTRUCTURE ONLY: CPU oracle for the BLS12-381 verification path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product (lodestar_amd, libblsgpu) never imports or links anything under oracle/.
"""
