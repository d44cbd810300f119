// Jupyter web app frontend: notebook table (polled with backoff), connect / start / stop / delete,
// notebook details (overview / events / logs / YAML), and the spawner dialog built from /api/config
// (MI355X GPU counts from the amd.com/gpu vendor, workspace + data volumes new or existing,
// affinity / toleration groups, PodDefault configurations, shared memory).
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
    const e = kf.esc;
    tr.innerHTML = `<td>${kf.statusCell(nb.status)}</td><td><a class="name">${e(nb.name)}</a></td><td>${e(nb.serverType)}</td><td>${e(nb.age)}</td>
      <td title="${e(nb.image)}">${e(nb.shortImage)}</td><td>${e(nb.gpus.count || 0)}</td><td>${e(nb.cpu)}</td><td>${e(nb.memory)}</td>
      <td>${e((nb.volumes || []).join(", "))}</td>`;
    tr.querySelector("a.name").addEventListener("click", () => showDetails(ns, nb.name));
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

  // notebook page: overview / events / logs / YAML (JWA frontend pages/notebook-page)
  function showDetails(ns, name) {
    const base = `/api/namespaces/${ns}/notebooks/${name}`;
    const e = kf.esc;
    return kf.details(`Notebook ${ns}/${name}`, [
      { name: "Overview", render: async () => {
        const nb = (await kf.call("GET", base)).notebook;
        const spec = ((nb.spec || {}).template || {}).spec || {};
        const c = (spec.containers || [])[0] || {};
        const lim = (c.resources || {}).limits || {}, req = (c.resources || {}).requests || {};
        const ann = (nb.metadata || {}).annotations || {};
        const st = nb.status || {};
        return kf.kvTable([
          ["Name", nb.metadata.name], ["Namespace", nb.metadata.namespace],
          ["Created", nb.metadata.creationTimestamp], ["Image", c.image],
          ["Server type", ann["notebooks.kubeflow.org/server-type"] || "jupyter"],
          ["CPU (request / limit)", `${req.cpu || "-"} / ${lim.cpu || "-"}`],
          ["Memory (request / limit)", `${req.memory || "-"} / ${lim.memory || "-"}`],
          ["MI355X GPUs", lim["amd.com/gpu"] || "0"], ["Allocated GPU ids", st.gpus || "-"],
          ["Volumes", (spec.volumes || []).map((v) => v.name).join(", ")],
          ["Ready replicas", st.readyReplicas || 0],
          ["Last activity", ann["notebooks.kubeflow.org/last-activity"] || "-"],
          ["Stopped", ann["kubeflow-resource-stopped"] || "no"],
        ]) + (st.gpuReadiness ? `<h3>GPU readiness op</h3><pre class="yaml">${e(kf.toYaml(st.gpuReadiness))}</pre>` : "") +
          `<h3>Conditions</h3>${kf.kvTable((st.conditions || []).map((x) => [x.type, `${x.status} ${x.reason || ""} ${x.message || ""}`]))}`;
      } },
      { name: "Events", render: async () => kf.eventsTable((await kf.call("GET", `${base}/events`)).events) },
      { name: "Logs", render: async () => {
        const pod = (await kf.call("GET", `${base}/pod`)).pod;
        const logs = (await kf.call("GET", `${base}/pod/${pod.metadata.name}/logs`)).logs;
        return `<p class="muted">Pod ${e(pod.metadata.name)}</p><pre class="logs">${e(logs.join("\n"))}</pre>`;
      } },
      { name: "YAML", render: async () => `<pre class="yaml">${e(kf.toYaml((await kf.call("GET", base)).notebook))}</pre>` },
    ]);
  }

  // data volumes: rows of {type new|existing, name, size, mode, mount}
  function addDataVolume(existing) {
    const rowEl = document.createElement("div");
    rowEl.className = "datavol";
    const pvcs = existing || [];
    rowEl.innerHTML = `<select class="dv-type"><option value="new">new</option><option value="existing">existing</option></select>
      <input class="dv-name" placeholder="{notebook-name}-data" size="16">
      <select class="dv-existing" hidden>${pvcs.map((p) => `<option>${kf.esc(p.name)}</option>`).join("")}</select>
      <input class="dv-size" value="10Gi" size="5"><select class="dv-mode"><option>ReadWriteOnce</option><option>ReadWriteMany</option><option>ReadOnlyMany</option></select>
      <input class="dv-mount" placeholder="/home/jovyan/data" size="18"><button type="button" class="dv-rm">&times;</button>`;
    rowEl.querySelector(".dv-type").onchange = (ev) => {
      const ex = ev.target.value === "existing";
      rowEl.querySelector(".dv-existing").hidden = !ex;
      ["dv-name", "dv-size", "dv-mode"].forEach((c) => { rowEl.querySelector("." + c).hidden = ex; });
    };
    rowEl.querySelector(".dv-rm").onclick = () => rowEl.remove();
    $("f-datavols").append(rowEl);
  }

  function dataVolumes() {
    return [...$("f-datavols").querySelectorAll(".datavol")].map((r) => {
      const q = (c) => r.querySelector("." + c).value.trim();
      const mount = q("dv-mount") || "/home/jovyan/data";
      if (q("dv-type") === "existing") return { mount, existingSource: { persistentVolumeClaim: { claimName: q("dv-existing") } } };
      return { mount, newPvc: { metadata: { name: q("dv-name") || "{notebook-name}-data" },
                                spec: { resources: { requests: { storage: q("dv-size") } }, accessModes: [q("dv-mode")] } } };
    });
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
    const opts = (key) => ['<option value="none">None</option>'].concat(((config[key] || {}).options || [])
      .map((o) => `<option value="${kf.esc(o.configKey)}" ${o.configKey === (config[key] || {}).value ? "selected" : ""}>${kf.esc(o.displayName || o.configKey)}</option>`)).join("");
    $("f-affinity").innerHTML = opts("affinityConfig");
    $("f-toleration").innerHTML = opts("tolerationGroup");
  }

  async function openSpawner() {
    const ns = kf.namespace();
    const { poddefaults } = await kf.call("GET", `/api/namespaces/${ns}/poddefaults`);
    $("f-configs").innerHTML = poddefaults.map((pd) =>
      `<label class="muted"><input type="checkbox" value="${kf.esc(pd.label)}"> ${kf.esc(pd.desc)}</label><br>`).join("") || '<span class="muted">none</span>';
    let pvcs = [];
    try { pvcs = (await kf.call("GET", `/api/namespaces/${ns}/pvcs`)).pvcs; } catch (e) { /* optional */ }
    $("f-datavols").replaceChildren();
    $("f-add-vol").onclick = () => addDataVolume(pvcs);
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
      tolerationGroup: $("f-toleration").value || "none", affinityConfig: $("f-affinity").value || "none",
      shm: $("f-shm").checked,
      configurations: [...$("f-configs").querySelectorAll("input:checked")].map((i) => i.value),
      datavols: dataVolumes(),
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
