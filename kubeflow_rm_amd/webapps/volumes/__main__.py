from kubeflow_rm_amd.webapps import crud_backend
from kubeflow_rm_amd.webapps.volumes import create_app

if __name__ == "__main__":
    crud_backend.serve(create_app(), 5000)
