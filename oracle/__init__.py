"""CPU oracle for the DRT MI355X hot path — TEST INFRASTRUCTURE ONLY.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it, and only as the checker / the timed CPU baseline; the product path
(``denseretrievaltoolkits_amd``) never imports it and has no CPU fallback.
"""
