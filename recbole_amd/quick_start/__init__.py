from recbole_amd.quick_start.quick_start import objective_function, run_recbole

__all__ = ['run_recbole', 'objective_function']
