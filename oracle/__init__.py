"""CPU oracle package -- TEST INFRASTRUCTURE ONLY.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg;
never by the product package graphneuralnetwork_amd.
"""
