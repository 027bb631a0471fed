"""indy7_mpc_amd — MI355X-native batched SQP-MPC for the Indy7 arm.

Drop-in for the reference's OSQP SQP-MPC hot path (A2R-Lab/indy7-mpc src/osqp_solver.py,
src/osqp_sqp.py, src/osqp_mpc.py): same class names and call surfaces, computed by HIP
kernels for gfx950 behind the C-ABI in include/indy7_mpc.h.
"""
__version__ = "0.1.0"
