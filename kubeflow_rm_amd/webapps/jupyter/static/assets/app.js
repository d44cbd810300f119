// Jupyter web app frontend: notebook table (polled with backoff), connect / start / stop / delete,
// and the spawner dialog built from /api/config (MI355X GPU counts from the amd.com/gpu vendor).
(function () {
  "use strict";
  const $ = (id) => document.getElementById(id);
  let config = null, poller = null;

  async function loadNamespaces() {
    let namespaces = [];
    try { namespaces = (await kf.call("GET", "/api/namespaces")).namespaces; }
    catch (e) { namespaces = kf.namespace() ? [kf.namespace()] : []; }  // not cluster-wide: dashboard drives it
    const sel = $("ns");
    sel.innerHTML = namespaces.map((n) => `<option>${n}</option>`).join("");
    if (!kf.namespace() && namespaces.length) kf.setNamespace(namespaces[0]);
    sel.value = kf.namespace();
    sel.onchange = () => kf.setNamespace(sel.value);
  }

  function row(nb, ns) {
    const tr = kf.h("tr", {});
    const stopped = nb.status.phase === "stopped";
    tr.innerHTML = `<td>${kf.statusCell(nb.status)}</td><td>${nb.name}</td><td>${nb.serverType}</td><td>${nb.age}</td>
      <td title="${nb.image}">${nb.shortImage}</td><td>${nb.gpus.count || 0}</td><td>${nb.cpu}</td><td>${nb.memory}</td>
      <td>${(nb.volumes || []).join(", ")}</td>`;
    const td = kf.h("td", {});
    const connect = kf.h("button", { onclick: () => window.open(`/notebook/${ns}/${nb.name}/`) }, "Connect");
    if (nb.status.phase !== "ready") connect.disabled = true;
    td.append(connect,
      kf.h("button", { onclick: () => act("PATCH", ns, nb.name, { stopped: !stopped }) }, stopped ? "Start" : "Stop"),
      kf.h("button", { onclick: () => confirm(`Delete notebook ${nb.name}?`) && act("DELETE", ns, nb.name) }, "Delete"));
    tr.append(td);
    return tr;
  }

  async function refresh() {
    const ns = kf.namespace();
    if (!ns) return null;
    const { notebooks } = await kf.call("GET", `/api/namespaces/${ns}/notebooks`);
    const body = $("notebooks").querySelector("tbody");
    body.replaceChildren(...notebooks.map((nb) => row(nb, ns)));
    return notebooks.map((nb) => [nb.name, nb.status.phase]);
  }

  async function act(method, ns, name, body) {
    try { await kf.call(method, `/api/namespaces/${ns}/notebooks/${name}`, body); $("error").textContent = ""; }
    catch (e) { $("error").textContent = e.message; }
    poller.reset();
  }

  function fillSpawner() {
    const imgs = config.image.options || [];
    $("f-image").innerHTML = imgs.map((i) => `<option ${i === config.image.value ? "selected" : ""}>${i}</option>`).join("");
    $("f-cpu").value = config.cpu.value; $("f-mem").value = config.memory.value;
    const gpu = config.gpus.value;
    const counts = gpu.options || ["none", "1", "2", "4", "8"];
    $("f-gpus").innerHTML = counts.map((c) => `<option ${c === gpu.num ? "selected" : ""}>${c}</option>`).join("");
    $("f-shm").checked = !!config.shm.value;
  }

  async function openSpawner() {
    const ns = kf.namespace();
    const { poddefaults } = await kf.call("GET", `/api/namespaces/${ns}/poddefaults`);
    $("f-configs").innerHTML = poddefaults.map((pd) =>
      `<label class="muted"><input type="checkbox" value="${pd.label}"> ${pd.desc}</label><br>`).join("") || '<span class="muted">none</span>';
    $("f-error").textContent = "";
    $("spawner").showModal();
  }

  async function submit(ev) {
    if (ev.submitter && ev.submitter.value !== "ok") return;
    ev.preventDefault();
    const ns = kf.namespace(), name = $("f-name").value;
    const gpus = $("f-gpus").value;
    const custom = $("f-custom").value.trim();
    const body = {
      name, namespace: ns, serverType: $("f-type").value,
      image: custom || $("f-image").value, customImage: !!custom, imagePullPolicy: config.imagePullPolicy.value,
      cpu: $("f-cpu").value, memory: $("f-mem").value,
      gpus: gpus === "none" ? { num: "none" } : { num: gpus, vendor: config.gpus.value.vendor },
      tolerationGroup: "none", affinityConfig: "none", shm: $("f-shm").checked,
      configurations: [...$("f-configs").querySelectorAll("input:checked")].map((i) => i.value),
      datavols: [],
    };
    if ($("f-ws").checked) {
      body.workspace = JSON.parse(JSON.stringify(config.workspaceVolume.value));
    }
    try { await kf.call("POST", `/api/namespaces/${ns}/notebooks`, body); $("spawner").close(); poller.reset(); }
    catch (e) { $("f-error").textContent = e.message; }
  }

  async function main() {
    try {
      config = (await kf.call("GET", "/api/config")).config;
      fillSpawner();
      await loadNamespaces();
    } catch (e) { $("error").textContent = e.message; }
    $("new").onclick = openSpawner;
    $("form").addEventListener("submit", submit);
    poller = new kf.Poller(refresh);
    kf.onNamespace((ns) => { $("ns").value = ns; poller.reset(); });
    poller.start();
  }
  main();
})();
