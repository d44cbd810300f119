"""Preload module for tests/test_zygote.py: leaves a (named) native thread running, as a BLAS or
runtime pool would."""
import threading
import time

threading.Thread(target=time.sleep, args=(60,), name="sleeper", daemon=True).start()
