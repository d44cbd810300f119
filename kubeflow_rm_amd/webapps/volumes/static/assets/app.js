// Volumes web app frontend: PVC list (polled) with the notebooks using each one, create / delete,
// volume details (overview / events / pods using it / YAML) and the PVCViewer (file browser)
// lifecycle: browse -> create viewer -> open its URL when ready.
(function () {
  "use strict";
  const $ = (id) => document.getElementById(id);
  let poller = null;
  async function namespaces() {
    let list = [];
    try { list = (await kf.call("GET", "/api/namespaces")).namespaces; } catch (e) { list = kf.namespace() ? [kf.namespace()] : []; }
    $("ns").innerHTML = list.map((n) => `<option>${n}</option>`).join("");
    if (!kf.namespace() && list.length) kf.setNamespace(list[0]);
    $("ns").value = kf.namespace();
    $("ns").onchange = () => kf.setNamespace($("ns").value);
  }
  async function act(method, path, body) {
    try { await kf.call(method, path, body); $("error").textContent = ""; } catch (e) { $("error").textContent = e.message; }
    poller.reset();
  }
  // volume page: overview / events / pods / YAML (VWA frontend pages/volume-details-page)
  function showDetails(ns, name) {
    const base = `/api/namespaces/${ns}/pvcs/${name}`;
    const e = kf.esc;
    return kf.details(`Volume ${ns}/${name}`, [
      { name: "Overview", render: async () => {
        const pvc = (await kf.call("GET", base)).pvc;
        const spec = pvc.spec || {}, st = pvc.status || {};
        return kf.kvTable([
          ["Name", pvc.metadata.name], ["Namespace", pvc.metadata.namespace], ["Created", pvc.metadata.creationTimestamp],
          ["Phase", st.phase || "-"], ["Requested", ((spec.resources || {}).requests || {}).storage || "-"],
          ["Capacity", (st.capacity || {}).storage || "-"], ["Access modes", (spec.accessModes || []).join(", ")],
          ["Storage class", spec.storageClassName || "(default)"], ["Volume", spec.volumeName || "-"],
        ]);
      } },
      { name: "Events", render: async () => kf.eventsTable((await kf.call("GET", `${base}/events`)).events) },
      { name: "Pods", render: async () => {
        const pods = (await kf.call("GET", `${base}/pods`)).pods;
        if (!pods.length) return '<p class="muted">Not mounted by any pod.</p>';
        return kf.kvTable(pods.map((p) => [p.metadata.name, `${(p.status || {}).phase || ""} on ${(p.spec || {}).nodeName || "-"}`]));
      } },
      { name: "YAML", render: async () => `<pre class="yaml">${e(kf.toYaml((await kf.call("GET", base)).pvc))}</pre>` },
    ]);
  }

  async function refresh() {
    const ns = kf.namespace();
    if (!ns) return null;
    const { pvcs } = await kf.call("GET", `/api/namespaces/${ns}/pvcs`);
    $("rows").querySelector("tbody").replaceChildren(...pvcs.map((p) => {
      const tr = kf.h("tr", {});
      const e = kf.esc;
      tr.innerHTML = `<td>${kf.statusCell(p.status)}</td><td><a class="name">${e(p.name)}</a></td><td>${e(p.age)}</td><td>${e(p.capacity)}</td>
        <td>${e((p.modes || []).join(", "))}</td><td>${e(p.class || "")}</td><td>${e(p.notebooks.join(", "))}</td>`;
      tr.querySelector("a.name").addEventListener("click", () => showDetails(ns, p.name));
      const v = p.viewer || {};
      const browse = kf.h("button", { onclick: () => (v.status === "ready" && v.url ? window.open(v.url)
        : v.status === "uninitialized" ? act("POST", `/api/namespaces/${ns}/viewers`, { name: p.name }) : null) },
        v.status === "ready" ? "Open browser" : v.status === "uninitialized" ? "Browse" : `Browser ${v.status}`);
      const close = kf.h("button", { onclick: () => act("DELETE", `/api/namespaces/${ns}/viewers/${p.name}`) }, "Close browser");
      close.disabled = v.status === "uninitialized";
      const del = kf.h("button", { onclick: () => confirm(`Delete volume ${p.name}?`) && act("DELETE", `/api/namespaces/${ns}/pvcs/${p.name}`) }, "Delete");
      tr.append(kf.h("td", {}, browse, close, del));
      return tr;
    }));
    return pvcs.map((p) => [p.name, p.status.phase, (p.viewer || {}).status]);
  }
  async function open() {
    let classes = [], def = "";
    try { classes = (await kf.call("GET", "/api/storageclasses")).storageClasses; def = (await kf.call("GET", "/api/storageclasses/default")).defaultStorageClass; } catch (e) { /* not cluster-readable */ }
    $("f-class").innerHTML = `<option value="{empty}">(default${def ? ": " + def : ""})</option><option value="{none}">(none)</option>` +
      classes.map((c) => `<option>${c}</option>`).join("");
    $("dlg").showModal();
  }
  async function submit(ev) {
    if (ev.submitter && ev.submitter.value !== "ok") return;
    ev.preventDefault();
    const ns = kf.namespace();
    const body = { name: $("f-name").value, size: $("f-size").value, mode: $("f-mode").value, class: $("f-class").value, type: "empty" };
    try { await kf.call("POST", `/api/namespaces/${ns}/pvcs`, body); $("dlg").close(); poller.reset(); }
    catch (e) { $("f-error").textContent = e.message; }
  }
  (async function main() {
    await namespaces();
    $("new").onclick = open;
    $("form").addEventListener("submit", submit);
    poller = new kf.Poller(refresh);
    kf.onNamespace((ns) => { $("ns").value = ns; poller.reset(); });
    poller.start();
  })();
})();
