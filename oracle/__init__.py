"""Oracle package -- TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's algorithms used to check the HIP path.  Importable only from
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never from the product
(``modelopt_amd``).
"""
