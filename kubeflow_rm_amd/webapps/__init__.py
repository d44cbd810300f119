"""CRUD web apps and the central dashboard backend (T5), Flask-based.

* :mod:`.crud_backend` — shared library: app factory, authn (user header), authz
  (SubjectAccessReview per Kubernetes call), CSRF double-submit cookie, probes, SPA serving,
  error handlers, status phases, Kubernetes API wrappers (on kubeflow_rm_amd.client).
* :mod:`.jupyter` — Jupyter web app (JWA): notebook spawner with MI355X GPU selection.
* :mod:`.tensorboards` — TensorBoards web app (TWA).
* :mod:`.volumes` — Volumes web app (VWA) with PVCViewer management.
* :mod:`.dashboard` — central dashboard backend (workgroups via KFAM, links, metrics) + shell UI.

Each app runs as ``python -m kubeflow_rm_amd.webapps.<app>`` (env: APP_PREFIX, PORT or
KFAMD_CONTAINER_PORTS, USERID_HEADER/USERID_PREFIX, APP_DISABLE_AUTH, APP_SECURE_COOKIES,
BACKEND_MODE=dev|prod).
"""
